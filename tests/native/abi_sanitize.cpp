// Host sanitizer driver for libmerging_hip's host code (test infrastructure):
// tests/test_sanitizers.py compiles merging_hip.hip with -Xarch_host -fsanitize=address,undefined
// and links this file. Every entry point's argument validation and the host helpers run without
// a GPU (nothing here launches a kernel); any sanitizer report aborts the run.
#include <cstdio>
#include <cstring>
#include <vector>

#include "merging_hip.h"

static int expect_error(int rc, const char* what) {
  if (rc == 0 || std::strlen(mg_last_error()) == 0) {
    std::printf("FAIL: %s was accepted\n", what);
    return 1;
  }
  return 0;
}

// The host step path (ABI 20) actually runs: 130 envs (a partial last mask word) in exactly sized
// heap arrays, 3,000 autoreset steps with every optional output, None / invalid actions and
// observe / reset calls in between, so the sanitizers see every access the host loop makes.
static int host_step_run(const mg_params& p) {
  const int64_t n = 130, words = (n + 63) / 64;
  std::vector<double> p1(n), v1(n), p2(n), v2(n), r1(n), r2(n);
  std::vector<uint16_t> tf(n);
  std::vector<float> obs(n * MG_OBS_DIM), rew(n * 2), fobs(n * MG_OBS_DIM);
  std::vector<uint8_t> flags(n * 4), done(n), coll(n), mask(n);
  std::vector<uint64_t> dm(words), wm(words);
  std::vector<mg_episode_stats> st(n);
  std::vector<mg_rec64> rec(n);
  std::vector<int8_t> a1(n), a2(n);
  int32_t err = 0;
  mg_state s{p1.data(), v1.data(), p2.data(), v2.data(), r1.data(), r2.data(), tf.data()};
  mg_outputs of{};
  of.obs = obs.data();
  of.rew = rew.data();
  of.done_mask = dm.data();
  of.final_obs = fobs.data();
  of.error = &err;
  of.won_mask = wm.data();
  of.flags = flags.data();
  mg_outputs ob{};  // the byte arrays and the fp64 record instead of the interleaved step record
  ob.done = done.data();
  ob.coll = coll.data();
  ob.rec64 = rec.data();
  ob.error = &err;
  mg_stats ms{st.data()};
  int bad = 0;
  if (mg_host_reset(&p, &s, nullptr, &of, n) != 0) ++bad;
  uint32_t episodes = 0;
  for (int k = 0; k < 3000; ++k) {
    for (int64_t i = 0; i < n; ++i) {
      a1[i] = static_cast<int8_t>((k * 7 + i) % 5);
      a2[i] = static_cast<int8_t>((k + 3 * i) % 6 - 1);  // -1 = None
    }
    if (k % 500 == 499) a1[k % n] = 9;  // the reference's KeyError path
    const bool f64 = k % 3 == 0;
    if (mg_host_step(&p, &s, a1.data(), a2.data(), f64 ? &ob : &of, &ms, n, f64 ? 0u : MG_AUTORESET) != 0) ++bad;
    if (k % 500 == 499 && err != 1) ++bad;
    err = 0;
    if (k % 400 == 0) {
      for (int64_t i = 0; i < n; ++i) mask[i] = static_cast<uint8_t>(i % 3 == 0);
      if (mg_host_observe(&p, &s, &ob, n) != 0 || mg_host_reset(&p, &s, mask.data(), &ob, n) != 0) ++bad;
    }
  }
  for (int64_t i = 0; i < n; ++i) episodes += st[i].episodes;
  if (episodes == 0) ++bad;
  std::printf("host step run: %u episodes finished\n", episodes);
  return bad;
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
  bad += host_step_run(p);
  std::printf("abi sanitizer run: %d failures\n", bad);
  return bad;
}
