"""Phase-clock instrumentation of the h-DQN / config-5 kernels (a diagnostic build, never shipped):
each wave of blocks 0..63 stamps s_memtime at the start of every phase and just before the phase's
closing barrier into a device array that mg_debug_clocks copies out. Applied as text edits to a
source file (the shipped one or an older one):

    python tools/clk_variant.py SRC OUT.so [0|1|base|q5|q5base]

(0 / 1 / base: the h-DQN kernel's phases, with the round-5 or round-4 forward marks; q5 / q5base:
the config-5 kernel's, working tree or round-4 source.)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "merging-gym_amd"))
from merging_gym import build  # noqa: E402

HDR = '''
__device__ unsigned g_mg_clk[64 * 8 * 64 * 16];
// event ev of phase p of this wave (0: phase start, 1: before the closing barrier, 2..15: marks)
#define MG_CLK(ev) do { if (blockIdx.x < 64 && (threadIdx.x & 63) == 0 && p < 64) \\
  g_mg_clk[((blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + p) * 16 + (ev)] = static_cast<unsigned>(__builtin_amdgcn_s_memtime()); } while (0)
extern "C" int mg_debug_clocks(void* dst) { return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mg_clk), sizeof(g_mg_clk)); }
'''
# config-5 (qnet_rollout_ws_kernel): phase marks of both roles, and a mark pair around each forward
# of the Q-net waves (the k-th forward of a phase: 2 + k before, 8 + k after, k < 6)
Q5_EDITS = [
    ("""    __syncthreads();
    for (int p = 0; p < phases; ++p) {
      if constexpr (OPP == 3) {""",
     """    __syncthreads();
    for (int p = 0; p < phases; ++p) {
      MG_CLK(0);
      int fidx = 0;
      if constexpr (OPP == 3) {"""),
    ("""        __syncthreads();
        continue;
      }""",
     """        MG_CLK(1);
        __syncthreads();
        continue;
      }""", 2),
    ("""            qnet_mlp_swp_nc(net, input(r), input(32 + r), q, col_tiles(cnt));""",
     """            if (fidx < 6) MG_CLK(2 + fidx);
            qnet_mlp_swp_nc(net, input(r), input(32 + r), q, col_tiles(cnt));
            asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[4]));
            if (fidx < 6) MG_CLK(8 + fidx);
            ++fidx;"""),
    ("""            qnet_mlp_swp_nc((OPP == 3 && opp) ? lds_net2 : lds_net, input(r), input(32 + r), q, col_tiles(cnt));""",
     """            if (fidx < 6) MG_CLK(2 + fidx);
            qnet_mlp_swp_nc((OPP == 3 && opp) ? lds_net2 : lds_net, input(r), input(32 + r), q, col_tiles(cnt));
            asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[4]));
            if (fidx < 6) MG_CLK(8 + fidx);
            ++fidx;"""),
]
Q5_BASE_EDITS = [
    ("""    __syncthreads();
    for (int p = 0; p < phases; ++p) {
      if (p < 2 * R.num_steps) {""",
     """    __syncthreads();
    for (int p = 0; p < phases; ++p) {
      MG_CLK(0);
      if (p < 2 * R.num_steps) {"""),
    ("""            qnet_forward_swp(OPP == 3 ? lds_net2 : lds_net, tile, row0, true, q);""",
     """            MG_CLK(2 + 2 * tt);
            qnet_forward_swp(OPP == 3 ? lds_net2 : lds_net, tile, row0, true, q);
            asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[4]));
            MG_CLK(8 + 2 * tt);"""),
    ("""          else
            qnet_forward_swp(lds_net, tile, row0, false, q);""",
     """          else {
            MG_CLK(3 + 2 * tt);
            qnet_forward_swp(lds_net, tile, row0, false, q);
            asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[4]));
            MG_CLK(9 + 2 * tt);
          }"""),
]
Q5_COMMON = [
    ("""      __syncthreads();
    }
    return;
  }
  // env lane:""",
     """      MG_CLK(1);
      __syncthreads();
    }
    return;
  }
  // env lane:"""),
    ("""  for (int p = 0; p < phases; ++p) {
    if (p > 0) {
      const int g = (p - 1) & 1, t = (p - 1) >> 1;
      const int local0""",
     """  for (int p = 0; p < phases; ++p) {
    MG_CLK(0);
    if (p > 0) {
      const int g = (p - 1) & 1, t = (p - 1) >> 1;
      const int local0"""),
    ("""    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kIlp; ++j) {
    const int la""",
     """    MG_CLK(1);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kIlp; ++j) {
    const int la"""),
]
# the round-5 h-DQN Q-net waves' passes (not kept): a mark pair around each forward (2 + 2 stage +
# chunk parity before, 8 + ... after)
NEW_EDITS = [
    ("""        if (glob)
          qnet_mlp_nc<kQGlobalAhead>(qnet_global(stage == 1 ? R.meta_op : R.lower_op), x0, x1, q, col_tiles(cnt));
        else
          qnet_mlp_swp_nc(stage == 2 ? lds_lower : lds_meta, x0, x1, q, col_tiles(cnt));""",
     """        MG_CLK(2 + 2 * stage + (c0 > 0));
        if (glob)
          qnet_mlp_nc<kQGlobalAhead>(qnet_global(stage == 1 ? R.meta_op : R.lower_op), x0, x1, q, col_tiles(cnt));
        else
          qnet_mlp_swp_nc(stage == 2 ? lds_lower : lds_meta, x0, x1, q, col_tiles(cnt));
        asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[4]));
        MG_CLK(8 + 2 * stage + (c0 > 0));"""),
]
# the round-4 Q-net waves: marks around its four forwards (2/8 meta, 4/10 opponent meta, 6/12 lower,
# 7/13 opponent lower: the same slots as NEW_EDITS' stages)
BASE_EDITS = [
    ("""        float q[8];
        qnet_mlp_swp(lds_meta, x0, x1, q);
        gstar = argmax_first(q, R.num_goals);""",
     """        float q[8];
        MG_CLK(2);
        qnet_mlp_swp(lds_meta, x0, x1, q);
        asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]));
        MG_CLK(8);
        gstar = argmax_first(q, R.num_goals);"""),
    ("""          gop_star = argmax_first(q, R.num_goals);""",
     """          asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]));
          MG_CLK(10);
          gop_star = argmax_first(q, R.num_goals);"""),
    ("""          if constexpr (OPP == 3)
            qnet_mlp<kQGlobalAhead>(qnet_global(R.meta_op), x0, x1, q);  // the opponent's own Goal_DQN (:267)""",
     """          MG_CLK(4);
          if constexpr (OPP == 3)
            qnet_mlp<kQGlobalAhead>(qnet_global(R.meta_op), x0, x1, q);  // the opponent's own Goal_DQN (:267)"""),
    ("""        float q[8];
        qnet_mlp_swp(lds_lower, qnet_input_goal(""",
     """        float q[8];
        MG_CLK(6);
        qnet_mlp_swp(lds_lower, qnet_input_goal("""),
    ("""        b_act[j] = static_cast<uint8_t>(argmax_first(q, MG_NUM_ACTIONS));""",
     """        asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]));
        MG_CLK(12);
        b_act[j] = static_cast<uint8_t>(argmax_first(q, MG_NUM_ACTIONS));"""),
    ("""          const bf16x8 x1 = qnet_input_goal(tile + (row0 + 32 + r) * kObs, b_gop[row0 + 32 + r], h, true);""",
     """          const bf16x8 x1 = qnet_input_goal(tile + (row0 + 32 + r) * kObs, b_gop[row0 + 32 + r], h, true);
          MG_CLK(7);"""),
    ("""          b_aop[j] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));""",
     """          asm volatile("" :: "v"(qo[0]), "v"(qo[1]), "v"(qo[2]));
          MG_CLK(13);
          b_aop[j] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));"""),
]
# the h-DQN Q-net waves as kept in round 5 (opponent meta-net pass compacted): a mark at each
# boundary of the phase's segments -- 2 / 8 around the meta forward (its inputs before 2), 3 after
# the goal logic, 9 after the opponent meta pass, 6 / 12 around the lower forward, 7 / 13 around the
# opponent's lower forward
NOW_EDITS = [
    ("""        float q[8];
        qnet_mlp_swp(lds_meta, x0, x1, q);
        gstar = argmax_first(q, R.num_goals);""",
     """        float q[8];
        MG_CLK(2);
        qnet_mlp_swp(lds_meta, x0, x1, q);
        asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]));
        MG_CLK(8);
        gstar = argmax_first(q, R.num_goals);"""),
    ("""      int gop_t = 0;
      if constexpr (kOpNets) {  // upper_op.choose_goal""",
     """      int gop_t = 0;
      MG_CLK(3);
      if constexpr (kOpNets) {  // upper_op.choose_goal"""),
    ("""        gop_t = fresh_op ? (dfo == kHGreedy ? gop_star : dfo) : gop_prev;
      }""",
     """        gop_t = fresh_op ? (dfo == kHGreedy ? gop_star : dfo) : gop_prev;
      }
      MG_CLK(9);"""),
    ("""        float q[8];
        qnet_mlp_swp(lds_lower, xe0, xe1, q);""",
     """        float q[8];
        MG_CLK(6);
        qnet_mlp_swp(lds_lower, xe0, xe1, q);"""),
    ("""        b_act[j] = static_cast<uint8_t>(argmax_first(q, MG_NUM_ACTIONS));""",
     """        asm volatile("" :: "v"(q[0]), "v"(q[1]), "v"(q[2]));
        MG_CLK(12);
        b_act[j] = static_cast<uint8_t>(argmax_first(q, MG_NUM_ACTIONS));"""),
    ("""          const bf16x8 x0 = xo0, x1 = xo1;""",
     """          const bf16x8 x0 = xo0, x1 = xo1;
          MG_CLK(7);"""),
    ("""          b_aop[j] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));""",
     """          asm volatile("" :: "v"(qo[0]), "v"(qo[1]), "v"(qo[2]));
          MG_CLK(13);
          b_aop[j] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));"""),
]
# the same segments for the lower passes listed by the env waves (r05zh): marks around the ego's and
# the opponent's listed forwards
LIST_EDITS = NOW_EDITS[:3] + [
    ("""          if (nqe > 0) {
            float q[8];""",
     """          MG_CLK(6);
          if (nqe > 0) {
            float q[8];"""),
    ("""          if (nqo > 0) {  // lower_op.choose_action""",
     """          MG_CLK(12);
          MG_CLK(7);
          if (nqo > 0) {  // lower_op.choose_action"""),
    ("""            if (lane < nqo) b_aop[row0 + loo] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));
          }""",
     """            if (lane < nqo) b_aop[row0 + loo] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));
          }
          MG_CLK(13);"""),
]
EDITS = [
    # h-DQN Q-net waves
    ("    for (int p = 0; p < phases; ++p) {\n      const int g = p & 1, t = p >> 1;\n      const int row0 = g * kHHalf + 64 * wave;",
     "    for (int p = 0; p < phases; ++p) {\n      MG_CLK(0);\n      const int g = p & 1, t = p >> 1;\n      const int row0 = g * kHHalf + 64 * wave;"),
    ("      __syncthreads();\n    }\n    return;\n  }\n  // ------------------------------------------------------------------ the env step",
     "      MG_CLK(1);\n      __syncthreads();\n    }\n    return;\n  }\n  // ------------------------------------------------------------------ the env step"),
    # h-DQN env waves
    ("  for (int p = 0; p < phases; ++p) {\n    if (p > 0 && ((p - 1) >> 1) < T) {",
     "  for (int p = 0; p < phases; ++p) {\n    MG_CLK(0);\n    if (p > 0 && ((p - 1) >> 1) < T) {"),
    ("    __syncthreads();\n  }\n  // both groups' last rows",
     "    MG_CLK(1);\n    __syncthreads();\n  }\n  // both groups' last rows"),
]


def main(src, out, marks="0"):
    s = open(src).read()
    s = s.replace('#include "merging_hip.h"\n', '#include "merging_hip.h"\n' + HDR, 1)
    sets = {"0": EDITS, "1": EDITS + NEW_EDITS, "base": EDITS + BASE_EDITS,
            "q5": Q5_COMMON + Q5_EDITS, "q5base": Q5_COMMON + Q5_BASE_EDITS, "hnow": EDITS + NOW_EDITS, "hlist": EDITS + LIST_EDITS}
    for e in sets[marks]:
        a, b, n = e if len(e) == 3 else (*e, 1)
        assert s.count(a) == n, a[:80]
        s = s.replace(a, b)
    tmp = out + ".hip"
    open(tmp, "w").write(s)
    try:
        subprocess.check_call([build.hipcc(), *build.HIPCC_FLAGS, "-I", build.INCLUDE, "-o", out, tmp])
    finally:
        os.unlink(tmp)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
