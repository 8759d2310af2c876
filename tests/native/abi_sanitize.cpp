// Host sanitizer driver for libmerging_hip's host code (test infrastructure):
// tests/test_sanitizers.py compiles merging_hip.hip with -Xarch_host -fsanitize=address,undefined
// and links this file. Every entry point's argument validation and the host helpers run without
// a GPU (nothing here launches a kernel); any sanitizer report aborts the run.
#include <cstdio>
#include <cstring>

#include "merging_hip.h"

static int expect_error(int rc, const char* what) {
  if (rc == 0 || std::strlen(mg_last_error()) == 0) {
    std::printf("FAIL: %s was accepted\n", what);
    return 1;
  }
  return 0;
}

int main() {
  int bad = 0;
  mg_params p;
  mg_params_default(&p);
  mg_params_default(nullptr);
  if (mg_abi_version() != MG_ABI_VERSION || p.timeout_steps != 2501) return 1;
  void* fake = reinterpret_cast<void*>(uintptr_t{1} << 20);  // never dereferenced
  mg_state s{};
  mg_outputs o{};
  bad += expect_error(mg_step(&p, &s, nullptr, nullptr, &o, nullptr, 16, 0, nullptr), "NULL state");
  bad += expect_error(mg_step(nullptr, &s, nullptr, nullptr, &o, nullptr, 16, 0, nullptr), "NULL params");
  mg_state sf{};
  double* d = static_cast<double*>(fake);
  sf.p1 = sf.v1 = sf.p2 = sf.v2 = sf.ret1 = sf.ret2 = d;
  sf.tf = static_cast<uint16_t*>(fake);
  bad += expect_error(mg_step(&p, &sf, nullptr, nullptr, &o, nullptr, 16, 0, nullptr), "NULL a1");
  bad += expect_error(mg_step(&p, &sf, static_cast<int8_t*>(fake), nullptr, &o, nullptr, -1, 0, nullptr), "n < 0");
  mg_outputs om{};
  om.obs = reinterpret_cast<float*>(static_cast<char*>(fake) + 4);
  bad += expect_error(mg_step_random(&p, &sf, nullptr, nullptr, &om, nullptr, 16, 0, 1, 0, 1, 0, nullptr),
                      "misaligned obs");
  mg_traj tj{};
  tj.flags = reinterpret_cast<uint8_t*>(static_cast<char*>(fake) + 2);
  bad += expect_error(mg_rollout_random(&p, &sf, &tj, nullptr, 16, 0, 1, 0, 4, 1, 0, nullptr), "misaligned flags");
  bad += expect_error(mg_rollout_qnet(&p, &sf, &tj, nullptr, 16, 0, 1, 0, 4, fake, 9, 0, 0, 0, nullptr, 0, nullptr),
                      "out_dim 9");
  mg_traj tq{};
  bad += expect_error(mg_rollout_qnet(&p, &sf, &tq, nullptr, 16, 0, 1, 0, 4, fake, 5, 0, 3, 0, nullptr, 0, nullptr),
                      "opponent net missing");
  bad += expect_error(mg_qnet_pack(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 10, 5, fake, nullptr),
                      "NULL weights");
  bad += expect_error(mg_qnet_forward(fake, static_cast<float*>(fake), 17, 0, static_cast<float*>(fake), 4, nullptr), "in_dim 17");
  mg_transitions tr{};
  bad += expect_error(mg_replay_store(static_cast<float*>(fake), static_cast<uint64_t*>(fake), 16, 22, &tr, 4, 1, 0,
                                      fake, 1 << 20, nullptr), "missing transitions");
  tr.obs_first = tr.obs = tr.rew = static_cast<float*>(fake);
  tr.a1 = static_cast<int8_t*>(fake);
  bad += expect_error(mg_replay_store(static_cast<float*>(fake), static_cast<uint64_t*>(fake), 16, 24, &tr, 4, 1, 0,
                                      fake, 1 << 20, nullptr), "row_floats 24 without goals");
  bad += expect_error(mg_replay_store(static_cast<float*>(fake), static_cast<uint64_t*>(fake), 16, 22, &tr, 4, 1, 0,
                                      fake, 8, nullptr), "short scratch");
  bad += expect_error(mg_replay_sample(static_cast<float*>(fake), static_cast<uint64_t*>(fake), 0, 22, 0, 0, 0,
                                       static_cast<float*>(fake), nullptr, 4, nullptr), "capacity 0");
  mg_traj tj0{};
  mg_hdqn_traj ht{};
  int8_t* g8 = static_cast<int8_t*>(fake);
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, nullptr, nullptr, 16, 0, 1, 0, 4, fake, 3, fake, 0,
                                      1ull << 31, 2, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr), "self-play without goal_op");
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, g8, nullptr, 16, 0, 1, 0, 4, fake, 3, fake, 0,
                                      1ull << 31, 3, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr),
                      "opponent_mode 3 without its nets");
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, g8, nullptr, 16, 0, 1, 0, 4, fake, 3, fake, 0,
                                      1ull << 31, 4, fake, fake, nullptr, nullptr, 0, 0, nullptr), "opponent_mode 4");
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, nullptr, nullptr, 16, 0, 1, 0, 4, fake, 3, fake, 0,
                                      1ull << 31, 0, nullptr, nullptr, static_cast<float*>(fake), nullptr, 16, 0, nullptr),
                      "ring without counter");
  if (mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, nullptr, nullptr, 0, 0, 1, 0, 4, fake, 3, fake, 0, 1ull << 31, 0,
                      nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr) != 0) bad += 1;  // empty batch
  mg_hdqn_traj htm{};
  htm.no_break = static_cast<uint64_t*>(fake);
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &htm, nullptr, g8, nullptr, nullptr, 16, 0, 1, 0, 4, fake, 3,
                                      fake, 0, 1ull << 31, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr),
                      "Goal_DQN outputs without ext_acc");
  bad += expect_error(mg_rollout_hdqn(&p, &sf, &tj0, &ht, nullptr, g8, nullptr, nullptr, 16, 0, 1, 0, 4, fake, 3, fake, 0,
                                      1ull << 31, 0, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr),
                      "h-DQN loop without MG_AUTORESET");
  bad += expect_error(mg_goal_status(nullptr, static_cast<double*>(fake), g8, 4, nullptr), "goal_status NULL");
  bad += expect_error(mg_rollout_random(&p, &sf, &tj0, nullptr, 16, 0, 1, 0, 65536, 1, 0, nullptr), "T > 65535");
  if (mg_replay_scratch_bytes(1 << 20, 16) != 8 + 1024 * 8 + 65536 * 4 + 1024 * 4) bad += 1;
  if (mg_qnet_packed_bytes() % 16 != 0) bad += 1;
  // empty batches return before any launch
  if (mg_step(&p, &sf, static_cast<int8_t*>(fake), nullptr, &o, nullptr, 0, 0, nullptr) != 0) bad += 1;
  if (mg_reset(&p, &sf, nullptr, &o, 0, nullptr) != 0) bad += 1;
  std::printf("abi sanitizer run: %d failures\n", bad);
  return bad;
}
