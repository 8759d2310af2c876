"""Builds tools/variants/lib_pclk.so, a stamped diagnostic copy of the uniform-wave config-5 kernel
with the persistent grid (r06ab: tools/variants/qnet_uniform_waves.patch plus the chunk loop of
qnet_uniform_waves_persistent_items.patch without its LDS item counter) for tools/uni_chunk_clk.py.
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
("""  for (int64_t chunk = blockIdx.x; chunk < chunks; chunk += gridDim.x) {
  const int64_t wbase = chunk * kQUniThreads + 64 * wave;""",
"""  int ci = 0;
  for (int64_t chunk = blockIdx.x; chunk < chunks; chunk += gridDim.x, ++ci) {
  MG_STAMP(32 + ci, 0, __builtin_amdgcn_s_memtime()); MG_STAMP(32 + ci, 12, __builtin_amdgcn_s_memrealtime());
  const int64_t wbase = chunk * kQUniThreads + 64 * wave;"""),
("""  const int wrows = wrem <= 0 ? 0 : (wrem < 64 ? static_cast<int>(wrem) : 64);
  for (int t = 0; t < R.num_steps; ++t) {
    // park""",
"""  const int wrows = wrem <= 0 ? 0 : (wrem < 64 ? static_cast<int>(wrem) : 64);
  MG_STAMP(32 + ci, 1, __builtin_amdgcn_s_memtime());
  for (int t = 0; t < R.num_steps; ++t) {
    // park"""),
("""  if (live[0]) store_env(R.S, wbase + lane, e[0]);
  }
}""",
"""  MG_STAMP(32 + ci, 2, __builtin_amdgcn_s_memtime());
  if (live[0]) store_env(R.S, wbase + lane, e[0]);
  MG_STAMP(32 + ci, 3, __builtin_amdgcn_s_memtime()); MG_STAMP(32 + ci, 13, __builtin_amdgcn_s_memrealtime());
  }
}"""),
]
for o,n in ed:
    assert s.count(o)==1, o
    s=s.replace(o,n)
p=ROOT+'/merging-gym_amd/csrc/.pclk.hip'
open(p,'w').write(s)
subprocess.run(["/opt/rocm/bin/hipcc","--offload-arch=gfx950","-O3","-std=c++17","-fPIC","-shared","-ffp-contract=off","-fno-fast-math","-w",'-DMG_SRC_SHA="pclk"',"-I",ROOT+"/include","-o",ROOT+"/tools/variants/lib_pclk.so",p],check=True)
os.remove(p)
