"""Builds tools/variants/lib_dclk.so, a stamped diagnostic copy of the uniform-wave config-5 kernel
with 64-env items (tools/variants/qnet_uniform_waves_persistent_items.patch) for tools/uni_wave_clk.py.
Reads the working-tree source, which must hold that kernel (apply the patch first); never shipped."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s=open(ROOT+'/merging-gym_amd/csrc/merging_hip.hip').read()
HDR = '''
__device__ unsigned g_mg_clk[64 * 8 * 64 * 16];
#define MG_STAMP(slot, ev, val) do { if (blockIdx.x < 64 && (threadIdx.x & 63) == 0 && (slot) < 64) \\
  g_mg_clk[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + (slot)) * 16 + (ev)] = static_cast<unsigned>(val); } while (0)
extern "C" int mg_debug_clocks(void* dst) { return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mg_clk), sizeof(g_mg_clk)); }
'''
anchor="constexpr int kQUniThreads = 512;"
s=s.replace(anchor, HDR+anchor,1)
ed=[
("""  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(R.net + kQNetBytes);
    for (int j = tid; j < kQ32NetBytes / 16; j += blockDim.x) reinterpret_cast<f32x4*>(lds_net)[j] = src[j];
  }
  __shared__ int next_item;""",
"""  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  MG_STAMP(0, 12, __builtin_amdgcn_s_memrealtime()); MG_STAMP(0, 0, __builtin_amdgcn_s_memtime());
  {
    const f32x4* src = reinterpret_cast<const f32x4*>(R.net + kQNetBytes);
    for (int j = tid; j < kQ32NetBytes / 16; j += blockDim.x) reinterpret_cast<f32x4*>(lds_net)[j] = src[j];
  }
  int nit = 0; unsigned busy = 0;
  __shared__ int next_item;"""),
("""  const int64_t wbase = (blockIdx.x + static_cast<int64_t>(item >> 3) * gridDim.x) * kQUniThreads + 64 * (item & 7);""",
"""  const unsigned it0 = static_cast<unsigned>(__builtin_amdgcn_s_memtime());
  if (nit == 0) { MG_STAMP(0, 1, it0); MG_STAMP(0, 13, __builtin_amdgcn_s_memrealtime()); }
  const int64_t wbase = (blockIdx.x + static_cast<int64_t>(item >> 3) * gridDim.x) * kQUniThreads + 64 * (item & 7);"""),
("""  if (live[0]) store_env(R.S, wbase + lane, e[0]);
  }
}""",
"""  if (live[0]) store_env(R.S, wbase + lane, e[0]);
  busy += static_cast<unsigned>(__builtin_amdgcn_s_memtime()) - it0; ++nit;
  }
  MG_STAMP(0, 2, __builtin_amdgcn_s_memtime()); MG_STAMP(0, 14, __builtin_amdgcn_s_memrealtime());
  MG_STAMP(0, 3, busy); MG_STAMP(0, 4, nit);
}"""),
]
for o,n in ed:
    assert s.count(o)==1, o
    s=s.replace(o,n)
p=ROOT+'/merging-gym_amd/csrc/.dclk.hip'
open(p,'w').write(s)
subprocess.run(["/opt/rocm/bin/hipcc","--offload-arch=gfx950","-O3","-std=c++17","-fPIC","-shared","-ffp-contract=off","-fno-fast-math","-w",'-DMG_SRC_SHA="dclk"',"-I",ROOT+"/include","-o",ROOT+"/tools/variants/lib_dclk.so",p],check=True)
os.remove(p)
