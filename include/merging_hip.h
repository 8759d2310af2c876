/*
 * merging_hip.h — C-ABI of libmerging_hip.so, the MI355X (gfx950) batched MergingEnv.
 *
 * The reference (YikangZhang1641/merging-gym) is pure Python and has no FFI. Its plugin
 * boundary is the gym.Env registered as "merging_env-v0" (merging_gym/__init__.py:3-6).
 * Each entry point below replaces one method of that env for a whole batch of envs held
 * as a struct-of-arrays in device memory; merging_gym/_native.py binds them with ctypes.
 *
 *   mg_step         replaces MergeEnv.step(action1, action2=None)   merging_env.py:138-195
 *                     (with action_to_acc :134-136 -> helper.mpc_1d helper.py:152-191,
 *                      observe :118-132, lon2coord :48-58, is_collided :198-206,
 *                      corners :232-239)
 *   mg_step_random  the same step, actions drawn on the device (Philox4x32-10); it replaces
 *                     the callers' env.action_space.sample() / np.random.randint(0, 5)
 *                     exploration branch (scripts/main.py:110, scripts/hdqn.py:175)
 *   mg_replay_store / mg_replay_sample / mg_replay_scratch_bytes: the DQN replay memory on the
 *                     device -- DQN.store_transition (scripts/main.py:115-119, hdqn.py:180-184)
 *                     for a whole batch of transitions, and learn()'s uniform minibatch draw
 *                     np.random.choice(MEMORY_CAPACITY, BATCH_SIZE) (main.py:130-131)
 *   mg_stats_reduce (ABI 20) the batch's episode-statistics records summed in a fixed order: the
 *                     running totals of the scripts' logging loops (hdqn.py:330-346, main.py:221-228)
 *   mg_reset        replaces MergeEnv.reset()                        merging_env.py:208-230
 *   mg_observe      replaces MergeEnv.observe() and is_collided()    merging_env.py:118-132,
 *                     :198-206 (no state change)
 *   mg_rollout_random  T steps of mg_step_random in one launch (trajectory outputs); it
 *                     replaces the callers' per-step collection loop (scripts/main.py:192-220)
 *   mg_rollout_qnet T steps with the epsilon-greedy DQN policy fused in (bf16 MFMA): replaces
 *                     DQN.choose_action (scripts/main.py:99-112, hdqn.py:165-177) + env.step
 *   mg_rollout_hdqn   T steps of hdqn.py's acting loop (meta-net goal, lower net on [goal] + state,
 *                     goal_status intrinsic reward) fused with the env step: replaces
 *                     Goal_DQN.choose_goal / HDQN.choose_action + env.step (hdqn.py:280-323)
 *   mg_qnet_pack / mg_qnet_forward / mg_qnet_packed_bytes / mg_qnet_fragments /
 *   mg_qnet_fragment_bytes: the Q-net Net (main.py:30-47,
 *                     hdqn.py:38-55) in the kernel's packed bf16 layout, and its forward pass
 *   mg_host_step / mg_host_reset / mg_host_observe (ABI 20): mg_step / mg_reset / mg_observe on
 *                     HOST memory, for the single env of BASELINE config 1 (the reference's CPU
 *                     MergeEnv, merging_env.py:118-230, driven one step at a time by
 *                     scripts/human_player.py:112-187 and the scripts' list API)
 *   mg_abi_version, mg_last_error, mg_build_info, mg_params_default, mg_time_next_launch: library plumbing
 *                     and profiling (no reference twin).
 *
 * Conventions
 *   - Every pointer inside mg_state / mg_outputs / mg_stats / action arrays is a DEVICE
 *     pointer owned by the caller (HOST pointers for the mg_host_* entry points). The library
 *     never allocates, frees or synchronises.
 *   - Calls are stream-ordered on `stream` (a hipStream_t, NULL = default stream) and
 *     return immediately. Return value: 0 on success, otherwise a hipError_t value
 *     (as int) and mg_last_error() describes it (thread-local). No exception crosses
 *     the ABI.
 *   - Arithmetic is IEEE fp64 with no contraction, like the reference's Python floats;
 *     the fp32 outputs are the fp64 results rounded once.
 */
#ifndef MERGING_HIP_H_
#define MERGING_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_ABI_VERSION 20
#define MG_OBS_DIM 10   /* merging_env.py:75 observation_shape = (10) */
#define MG_NUM_ACTIONS 5 /* merging_env.py:101-102 action_dict / Discrete(5) */
#define MG_ACTION_NONE (-1) /* action2=None: the constant-speed "L0" opponent, merging_env.py:152 */

/* Bits of mg_state.tf (one uint16 per env). The step count only decides the timeout (done from
 * step 2501, merging_env.py:141-143), so it saturates at 8191. */
#define MG_TF_STEPS_MASK 0x1FFFu  /* steps since reset, saturating at 8191 */
#define MG_TF_WINNER_SHIFT 13     /* 2 bits: 0 = None, 1 = ego, 2 = opponent (self.winner) */
#define MG_TF_WINNER_MASK 0x6000u
#define MG_TF_DONE 0x8000u        /* self.done */

/* Flags argument of mg_step / mg_step_random. */
#define MG_AUTORESET 0x1u /* gym.vector semantics: an env that is done after this step is reset
                             in place; obs receives the reset observation and
                             out->final_obs (if non-NULL) the terminal one */

/* Bits of mg_rec64.status (single-env drop-in path). */
#define MG_ST_DONE 0x1u
#define MG_ST_COLLISION 0x2u
#define MG_ST_R1_INT 0x4u /* reward1 is the Python int the reference returns (merging_env.py:168) */
#define MG_ST_R2_INT 0x8u /* reward2 likewise (merging_env.py:178) */
#define MG_ST_V1_INT 0x10u /* vel1 is int 0 from max(0, ...) (merging_env.py:149) */
#define MG_ST_V2_INT 0x20u /* vel2 likewise (merging_env.py:153) */

/* Environment constants, merging_env.py:22-46 and :101. Fill with mg_params_default(). */
typedef struct mg_params {
  double R;            /* 30000: arc radius                          merging_env.py:22 */
  double H;            /* 1000                                        merging_env.py:23 */
  double W;            /* 300                                         merging_env.py:23 */
  double dT;           /* 0.2 s per step                              merging_env.py:25 */
  double r_first;      /* 2.0  RFirst                                 merging_env.py:28 */
  double r_second;     /* 1.0  RSecond                                merging_env.py:29 */
  double r_collision;  /* -10  RCollision                             merging_env.py:30 */
  double vel_penalty;  /* 0.001                                       merging_env.py:31 */
  double time_penalty; /* 0                                           merging_env.py:32 */
  double start_point;  /* 50                                          merging_env.py:36 */
  double end_point;    /* 950 = H - 50                                merging_env.py:37 */
  double start_vel;    /* 20.0 (reset)                                merging_env.py:216-217 */
  double vel_ref;      /* 20.0 (reward reference speed)               merging_env.py:158-159 */
  double prediction_t; /* 3.0 MPC horizon                             merging_env.py:43 */
  double angle0;       /* atan2(H, R), host-precomputed               merging_env.py:49 */
  double action_speed[MG_NUM_ACTIONS]; /* {0,10,20,30,40}             merging_env.py:101 */
  int32_t veh_w;       /* 4  lateral box size                         merging_env.py:40,97 */
  int32_t veh_h;       /* 8  longitudinal box size                    merging_env.py:40,97 */
  int32_t timeout_steps; /* 2501: first step with time_stamp > 500    merging_env.py:141-143 */
  int32_t _pad;
  double inv_R;        /* 1 / R, rounded: the kernel divides by R (and by qp_nz) with an
                          FMA-corrected reciprocal multiply (still correctly rounded) */
  /* mpc_1d's QP (scripts/helper.py:152-191) as quadprog 0.1.11's qpgen2 (the Goldfarb-Idnani
   * dual method, reached through qpsolvers 1.8.0 at helper.py:182) runs it: P = R'R by LINPACK
   * dpofa, J = R^-1 by dpori, then for the one equality (normal n = A[1], b = vt - v0, its sign
   * folded into n when the residual is positive) d = J'n, z = J d, t = |b| / z'n and
   * u = 0 + t z; a residual |b| < vsmall counts as satisfied (u = 0). So u0 = (b / z'n) * z0
   * with the two constants below computed in that operation order by mg_params_default (ABI
   * 17; ABI <= 16 used Cholesky substitution, an ulp apart). Restated from the published
   * algorithm -- quadprog is not importable here, so bit parity with it is unpinned. */
  double qp_nz;        /* z'n = 90.0000000000015 (t = 3) */
  double qp_z0;        /* z[0] = 30.000000000000533 */
  double qp_inv_nz;    /* 1 / qp_nz, rounded */
  double qp_vsmall;    /* qpgen2's vsmall: the first 1e-60 * 2^k with 1 + 0.1 vsmall > 1 and
                          1 + 0.2 vsmall > 1 (1.4272476927059598e-15) */
} mg_params;

/* Per-env state, struct of arrays, n entries each (device pointers). */
typedef struct mg_state {
  double* p1;   /* state1['pos']  (ego) */
  double* v1;   /* state1['vel'] */
  double* p2;   /* state2['pos']  (opponent) */
  double* v2;   /* state2['vel'] */
  double* ret1; /* r1_accumulate */
  double* ret2; /* r2_accumulate */
  uint16_t* tf; /* step count | winner | done, see MG_TF_* */
} mg_state;

/* Packed fp64 record for the single-env (list API) path. */
typedef struct mg_rec64 {
  double obs[MG_OBS_DIM];
  double rew[2];
  double acc[2];  /* state1['acc'], state2['acc'] */
  double pos[2];
  double vel[2];
  double ret[2];
  uint32_t tf;
  uint32_t status; /* MG_ST_* */
} mg_rec64;

/* Outputs of one step. Any pointer may be NULL to skip that output. */
typedef struct mg_outputs {
  float* obs;           /* [n,10] fp32, 16-byte aligned */
  float* rew;           /* [n,2]  fp32, 8-byte aligned */
  uint8_t* done;        /* [n] 0/1 */
  uint8_t* coll;        /* [n] 0/1, info["collision"] */
  uint64_t* done_mask;  /* [ceil(n/64)] bit j of word w = done of env 64w+j */
  float* final_obs;     /* [n,10] written only for envs that finished (with MG_AUTORESET) */
  mg_rec64* rec64;      /* [n] fp64 record (single-env drop-in path) */
  int32_t* error;       /* [1] OR-ed with 1 (a1) / 2 (a2) when an action is outside the valid set.
                           Such an env is advanced exactly as far as the reference gets before its
                           action_dict[...] KeyError (merging_env.py:141-147, :152): the clock
                           always, the ego too when only a2 is invalid; nothing else is written. */
  uint64_t* won_mask;   /* [ceil(n/64)] bit = env.winner == 1 after this step (read before any
                           autoreset): main.py:209 stores a transition only when it is 0 */
  uint8_t* flags;       /* [n,4] interleaved a1, a2 (int8), done, collision (0/1), 4-byte aligned:
                           one 32-bit store per env instead of four byte stores. When set, done
                           and coll must be NULL, and so must mg_step_random's a1_out / a2_out
                           (the actions land here); mg_observe writes byte 3. Not with rec64. */
} mg_outputs;

/* Trajectory buffers of mg_rollout_random: the outputs of step t for env i sit at row
 * t * n + i. Any pointer may be NULL to skip that output. */
typedef struct mg_traj {
  float* obs;       /* [T, n, 10] fp32, 16-byte aligned (reset observation where autoreset fired) */
  float* rew;       /* [T, n, 2] fp32 */
  uint8_t* done;    /* [T, n] */
  uint8_t* coll;    /* [T, n] */
  int8_t* a1;       /* [T, n] actions drawn */
  int8_t* a2;       /* [T, n] (-1 = None) */
  float* final_obs; /* [T, n, 10] written only at rows whose env finished at that step */
  uint64_t* won_mask; /* [T, ceil(n/64)] as mg_outputs.won_mask, one bitmask per step */
  uint8_t* flags;   /* [T, n, 4] = (a1, a2, done, coll) interleaved, 4-byte aligned, or NULL. When
                       set, the four byte arrays above are ignored and each env-step's four bytes
                       leave as one 32-bit store (separate byte arrays cost the rollout ~5 %) */
} mg_traj;

/* A batch of transitions for the replay memory, T steps of n envs in [T, n, ...] layout (the
 * trajectory buffers of a rollout, or one step's outputs with T = 1). Transition (t, i) is
 *   s  = obs_first[i] (t = 0) or obs[t-1, i],   a = a1[t, i],   r = rew[t, i, 0] (the ego's),
 *   s' = final_obs[t, i] where done[t, i] (autoreset put the reset observation in obs), else obs[t, i]
 * -- exactly what the reference's loop hands store_transition (main.py:195-211).
 * Goal-augmented rows (hdqn.py's lower-level memory, :158 np.zeros((MEMORY_CAPACITY,
 * (NUM_STATES + 1) * 2 + 2)), :180-184, fed at :291-316 with goal_state = [goal] + state):
 * with goal != NULL a row is 24 floats [goal, s(10), a, r, next_goal, s'(10)]; reward != NULL
 * replaces rew[t, i, 0] (hdqn's intrinsic reward, :314). */
typedef struct mg_transitions {
  const float* obs_first;   /* [n, 10] observation before step 0 */
  const float* obs;         /* [T, n, 10] */
  const float* final_obs;   /* [T, n, 10] or NULL (then s' = obs even where done) */
  const int8_t* a1;         /* [T, n] (or NULL with flags) */
  const float* rew;         /* [T, n, 2] */
  const uint8_t* done;      /* [T, n] or NULL (never done; ignored with flags) */
  const uint64_t* won_mask; /* [T, ceil(n/64)] or NULL (nobody has won) */
  const float* goal;        /* [T, n] goal column of s, or NULL (22-float rows) */
  const float* next_goal;   /* [T, n] goal column of s' (required with goal) */
  const float* reward;      /* [T, n] r of the row, or NULL (r = rew[t, i, 0]) */
  const uint8_t* flags;     /* [T, n, 4] interleaved (a1, a2, done, coll) of mg_traj.flags, or NULL:
                               then a1 = flags[4 row], done = flags[4 row + 2] */
  const float* meta_goal;   /* (ABI 15) [T, n] or NULL: Goal_DQN's memory instead (hdqn.py:97-101,
                               stored at :325 once an inner loop broke): row [s', meta_goal, reward,
                               s'] with s' the next state (terminal where done) for the transitions
                               whose won_mask bit is CLEAR -- the mask then marks the steps that did
                               not end an inner loop (mg_hdqn_traj.no_break) and is required, as is
                               reward (the extrinsic reward, mg_hdqn_traj.ext_reward); 22-float rows,
                               goal NULL, skip_ego_won ignored */
} mg_transitions;

/* Completed-episode statistics of one env, updated when it finishes (MG_AUTORESET): the
 * quantities the reference's training scripts log per episode, summed over the env's episodes
 * (ABI 17). One 64-byte record per env, so a finishing env's read-modify-write stays within one
 * cache line: as separate arrays (ABI <= 7) those scattered updates cost the one-step kernel 12 %
 * of its time at 2^22 envs (tools/steady_probe.py).
 *   main.py:189-227   ep_reward sums the ego's reward only over steps after which
 *                     `env.winner is not 1` (:209-211); win_count counts `state[8] > state[3]`
 *                     on the observation the episode's LAST step acted on (`state = next_state`
 *                     is skipped at the :218-220 break), i.e. END_POINT - p2 > END_POINT - p1
 *                     in fp64 on the state before that step;
 *   hdqn.py:276-346   ep_reward is every step's reward (= r1_accumulate, :312); win_count tests
 *                     `state[8] > state[3]` on the terminal observation (state = next_state at
 *                     :320 before the break).
 * winner never returns to 1 once it is 2, and stays 1 once set, so main.py's filtered sum is
 * r1_accumulate as it stood before the step on which the ego arrived first (or the whole
 * r1_accumulate when it never did): the kernels keep that value in ret1_pending. */
typedef struct mg_episode_stats {
  double ret[2];        /* sum of completed-episode returns r{1,2}_accumulate (hdqn.py's ep_reward) */
  double ret_main;      /* sum of main.py's winner-filtered ep_reward */
  double ret1_pending;  /* scratch (per env): r1_accumulate before the current episode's ego-first
                           arrival step; read only while winner == 1 */
  uint32_t episodes;    /* completed episodes */
  uint32_t collisions;  /* of which ended in a collision */
  uint32_t ego_first;   /* of which the ego arrived first (winner == 1) */
  uint32_t steps;       /* total steps of the completed episodes */
  uint32_t win_main;    /* main.py:225's win test on the pre-terminal observation */
  uint32_t win_hdqn;    /* hdqn.py:342's win test on the terminal observation */
  double q_eval;        /* (ABI 20; reserved zero bytes until ABI 19) sum over the completed episodes
                           of the Q value the scripts log for each (q_eval_value): the fused policy
                           kernels add eval_net(state)[action] on the last step's input and action
                           (mg_rollout_qnet, main.py:221) or meta_eval_net(state)[goal] on the terminal
                           state and the goal chosen on it (mg_rollout_hdqn, hdqn.py:330); the kernels
                           without a net leave it unchanged */
} mg_episode_stats;

typedef struct mg_stats {
  mg_episode_stats* rec;  /* [n] records, or NULL: no statistics */
} mg_stats;

/* (ABI 20) The records of a batch summed: what the logging loops of scripts/hdqn.py:330-346 and
 * scripts/main.py:221-228 total over completed episodes: the per-rank contribution of the
 * multi-GPU statistics all-gather (merging_gym/distributed.py), 80 bytes. */
typedef struct mg_stats_totals {
  double ret[3];      /* sums of ret[0], ret[1], ret_main */
  double q_eval;      /* sum of q_eval */
  int64_t counts[6];  /* sums of episodes, collisions, ego_first, steps, win_main, win_hdqn */
} mg_stats_totals;

int mg_abi_version(void);
const char* mg_last_error(void);
/* (ABI 20) The compiler and HIP version the library was built with, e.g. for test logs. */
const char* mg_build_info(void);

/* Profiling hook: the next mg_step / mg_step_random / mg_rollout_random launch made by the calling thread records
 * start_event / stop_event (hipEvent_t created by the caller; either may be NULL) in its own
 * dispatch packet (hipExtLaunchKernel), so hipEventElapsedTime(start, stop) is the kernel's
 * duration without the launch gap. Consumed by that launch. Always returns 0. */
int mg_time_next_launch(void* start_event, void* stop_event);

/* Fills *p with the reference constants (merging_env.py:22-46, :101). Host only. */
void mg_params_default(mg_params* p);

/* One env step for n envs. a1[n] in {0..4}; a2[n] in {0..4, -1 = None} or a2 == NULL (all None).
 * Replaces MergeEnv.step (merging_env.py:138-195). */
int mg_step(const mg_params* params, const mg_state* state, const int8_t* a1, const int8_t* a2,
            const mg_outputs* out, const mg_stats* stats, int64_t n, uint32_t flags, void* stream);

/* As mg_step, with actions drawn on the device (ABI 12): w = word ((step_idx div 2) mod 4) of
 * Philox4x32-10 (key = seed, counter = (env_offset + env index, step_idx div 8)) -- one call
 * covers eight steps of a rollout, two draws per word; a shard of a larger batch passes its first
 * global env index as env_offset and draws the same actions it would draw unsharded. A draw of
 * m outcomes is floor(m w / 2^32); an odd step_idx draws from m w mod 2^32 instead (the first
 * draw's remainder). opponent_random != 0: m = 25, the pair x = draw, a1 = x / 5, a2 = x % 5;
 * else m = 5, a1 = draw, a2 None.
 * If a1_out / a2_out are non-NULL the actions used are written there (-1 for None). */
int mg_step_random(const mg_params* params, const mg_state* state, int8_t* a1_out,
                   int8_t* a2_out, const mg_outputs* out, const mg_stats* stats, int64_t n,
                   int64_t env_offset, uint64_t seed, uint64_t step_idx,
                   int32_t opponent_random, uint32_t flags, void* stream);

/* num_steps consecutive steps with device-drawn actions in ONE launch: identical results to
 * num_steps calls of mg_step_random with step_idx = first_step + t, output of step t written
 * to slice t of *traj. Each env stays in registers for the whole launch, so its state is read
 * and written once instead of once per step. Replaces the callers' collection loop around
 * MergeEnv.step (scripts/main.py:192-220, scripts/hdqn.py:288-323) for a random policy. */
int mg_rollout_random(const mg_params* params, const mg_state* state, const mg_traj* traj,
                      const mg_stats* stats, int64_t n, int64_t env_offset, uint64_t seed,
                      uint64_t first_step, int32_t num_steps, int32_t opponent_random,
                      uint32_t flags, void* stream);

/* ---- DQN policy (scripts/main.py:30-47 Net, :99-112 choose_action) ---------------------------
 * A packed Q-net is one device buffer of mg_qnet_packed_bytes() bytes (16-byte aligned) made by
 * mg_qnet_pack from the fp32 torch tensors fc1.weight [200,in], fc1.bias [200], fc2.weight
 * [100,200], fc2.bias [100], out.weight [out,100], out.bias [out] (device pointers, row-major).
 * Weights are stored as bf16; each fp32 bias as three bf16 parts (hi + mid + lo == bias exactly)
 * in padded K slots whose inputs are 1.0, so the matrix cores add it inside the K sum; hidden
 * sizes are the reference's 200 and 100; 1 <= in_dim <= 13, 1 <= out_dim <= 8. ABI 19: the buffer
 * holds two layouts of the same bf16 values -- first the operand fragments of the 16x16x32 forward
 * (self-play / other-net opponents, h-DQN, mg_qnet_forward), then the 32x32x16 layout of the
 * config-5 instances without a net opponent. */
size_t mg_qnet_packed_bytes(void);
int mg_qnet_pack(const float* fc1_w, const float* fc1_b, const float* fc2_w, const float* fc2_b,
                 const float* out_w, const float* out_b, int32_t in_dim, int32_t out_dim,
                 void* packed, void* stream);

/* The fragment-major copy of a packed net, mg_qnet_fragment_bytes() = mg_qnet_packed_bytes(). Since
 * ABI 19 the packed layout itself is fragment-major -- the MFMA operand fragments of one forward in
 * the order the kernel consumes them, each the 64 lanes' 16 bytes contiguous (1 KB; the four
 * layer-3 fragments 512 B) -- so this is a plain copy, kept for ABI-18 callers (ABI 18: a
 * separate 66-KB layout). mg_rollout_hdqn reads an opponent from another checkpoint
 * (opponent_mode 3) from global memory in this layout: a fragment load touches 8 cache lines.
 * fragments: 16-byte aligned device buffer. */
size_t mg_qnet_fragment_bytes(void);
int mg_qnet_fragments(const void* packed, void* fragments, void* stream);

/* q[n,8] fp32 = Net(x[n,in_dim]) with bf16 operands and fp32 accumulation (rows >= out_dim are
 * padding; in_dim is the net's, 1..13: 10 for main.py's Net on observations, 11 for hdqn.py's
 * lower-level Net on goal states [goal] + state, :145, :291). swap_halves != 0 (in_dim 10 only)
 * feeds the opponent's view x[5:] + x[:5] (main.py:199). */
int mg_qnet_forward(const void* packed, const float* x, int32_t in_dim, int32_t swap_halves, float* q,
                    int64_t n, void* stream);

/* num_steps steps in ONE launch with the epsilon-greedy Q-net policy computed on the device,
 * Philox4x32-10 draws with key = seed. The ego acts greedily (argmax of Q(obs), lowest index on
 * ties) when its explore draw e < greedy_threshold and at random otherwise -- greedy_threshold =
 * round(Phi(0.7) 2^32) reproduces `np.random.randn() <= EPISILO` (main.py:105).
 * opponent_mode 0 (None) and 1 (uniform) -- two draws per step (ABI 20): step k = first_step + t
 * of env gi = env_offset + i takes words (u0, u1) of counter (gi, k div 2) when k is even and
 * (u2, u3) when k is odd; e = the first, and the second w gives the random action floor(5 w / 2^32)
 * (mode 0, opponent None) or the pair x = floor(25 w / 2^32), a1 = x div 5 (used when exploring),
 * a2 = x mod 5 (the uniform opponent, mode 1).
 * opponent_mode 2 and 3 -- counter (gi, k): u0 / u1 the ego's explore draw / random action
 * floor(5 u1 / 2^32), u2 / u3 the opponent's with opp_greedy_threshold: the same net on the swapped
 * observation (2, Strategy_OP "selfplay", main.py:165-166),
 * or another packed net opp_net (same out_dim) on the swapped observation the same way (3,
 * main.py's default Strategy_OP "L1": a separately trained DQN as the opponent, :161-168, :199;
 * ABI 14; opp_net is ignored by the other modes). Outputs as mg_rollout_random
 * (traj->obs[t] = observation after step t, the network input of step t + 1). */
int mg_rollout_qnet(const mg_params* params, const mg_state* state, const mg_traj* traj,
                    const mg_stats* stats, int64_t n, int64_t env_offset, uint64_t seed,
                    uint64_t first_step, int32_t num_steps, const void* net, int32_t out_dim,
                    uint64_t greedy_threshold, int32_t opponent_mode,
                    uint64_t opp_greedy_threshold, const void* opp_net, uint32_t flags, void* stream);

/* ---- h-DQN acting loop (scripts/hdqn.py:280-323) ----------------------------------------------
 * The per-step outputs of mg_rollout_hdqn besides mg_traj, [T, n] fp32 each (NULL skips one):
 * exactly the goal columns and intrinsic reward hdqn.py's lower-level store_transition takes
 * (:291, :304, :314, :316) -- feed them to mg_replay_store as mg_transitions.goal / next_goal /
 * reward for the 24-float goal rows. */
typedef struct mg_hdqn_traj {
  float* goal;       /* goal of step t's goal state [goal] + state (:291) */
  float* next_goal;  /* goal Goal_DQN chose on step t's next state (:303; the terminal one at an
                        episode end), the row's next goal */
  float* reward;     /* 1.0 if next_goal == goal_status(state) else 0.0 (:314) */
  float* goal_op;    /* (optional, opponent_mode 2 / 3) the opponent's goal of step t, the
                        goal of its goal state [goal_op] + swapped state (:285, :299) */
  float* ext_reward; /* (optional, ABI 15) extrinsic reward summed since the inner loop began,
                        through step t (:286, :311-313): Goal_DQN's row reward at a break;
                        needs ext_acc */
  uint64_t* no_break; /* (optional, ABI 15) [T, ceil(n/64)] bit i of word t ceil(n/64) + i/64 set
                        where step t did not end the inner loop (:322): the rows Goal_DQN does not
                        store (mg_transitions.meta_goal) */
} mg_hdqn_traj;

/* num_steps steps of hdqn.py's inner loop in ONE launch (opponent L0 or uniform random): per env
 * and step, the lower-level Net (lower_net: in 11, out 5) acts epsilon-greedily on the goal
 * state [goal] + state, the env steps, Goal_DQN's meta-net (meta_net: in 10, out num_goals)
 * chooses the next goal epsilon-greedily on the next state, goal_status gives the intrinsic
 * reward, and a fresh goal is chosen when that goal is already reached or the episode ended
 * (:320-322, :278-283; reset_goal = the meta-net's argmax on the reset observation, which the
 * caller computes once). goal_status is evaluated on the fp64 x2 - x1 and v2 of the state (ABI 17;
 * see mg_goal_status). flags must include MG_AUTORESET (hdqn.py resets at every episode end, :277;
 * ABI 17 rejects a launch without it). goal [n] int8 holds each env's current goal across launches (< 0: none
 * yet -- chosen by the meta-net at the first step). Random draws: Philox4x32-10 with key seed,
 * counter (env_offset + i, first_step + t) for the action and next goal (x, y, z, w = explore,
 * action, explore, goal) and stream B, counter ((env_offset + i) ^ 2^63, c), for a fresh goal's
 * explore / goal draws of step k: with the uniform opponent (mode 1) words (x, y) of c = k, its
 * action from z; otherwise (ABI 20) one call per two steps, c = k div 2, words (x, y) on even k
 * and (z, w) on odd k. A launch's first fresh goals use step first_step - 1.
 * Greedy when the explore draw < greedy_threshold (np.random.randn() <= EPISILO, :84, :168).
 * traj as mg_rollout_qnet; opponent_mode 0 (None, Strategy_OP "L0", :261, :294-296), 1 (uniform),
 * 2 (Strategy_OP "selfplay", :262-264: upper_op = upper, lower_op = lower, so the same two
 * nets) or 3 (any other Strategy_OP, :265-268: upper_op / lower_op loaded from another h-DQN
 * checkpoint -- opp_meta_net / opp_lower_net, the mg_qnet_fragments copies of its packed nets
 * (ABI 18; packed nets until ABI 17), 16-byte aligned, ignored by the other modes; ABI 16. Four
 * nets exceed one CU's LDS, so the opponent's two are read from global memory, where they stay
 * L2-resident): the opponent's goal is chosen by its
 * meta-net on the swapped state
 * state[5:] + state[:5] at every outer-loop iteration (:285 -- the launch's first step when
 * goal_op[i] < 0, and the step after a break: the ego's goal reached or the episode ended) and
 * kept in between; its action is its lower net's epsilon-greedy choice on
 * [goal_op] + swapped state every step (:299-300). Its draws: counter
 * ((env_offset + i) ^ 2^62, first_step + t), x explore and y action of step t, z explore and
 * w goal of a fresh opponent goal at step t + 1 (the launch's first at step first_step - 1).
 * goal_op [n] int8 (required for modes 2 and 3, else ignored) holds each env's opponent goal across
 * launches like goal. ext_acc [n] double (required with htraj->ext_reward or no_break, ABI 15)
 * holds each env's extrinsic reward since its inner loop began, across launches (0 at a break);
 * whenever it is given the sums are kept, with or without those outputs (ABI 17).
 * ring_rows (optional, 16-byte aligned [ring_capacity, 24] fp32, with ring_counter: one device
 * uint64): the launch also appends every transition to hdqn.py's lower-level memory
 * (HDQN.store_transition, :316, which stores them all) -- row [goal, s, a, r, next_goal, s'] of
 * (t, i) at slot (counter + t n + i) % ring_capacity, exactly what mg_replay_store with
 * skip_ego_won = 0 writes from this launch's outputs (only the newest ring_capacity rows when
 * more are appended), then counter += T n. No scan is needed since every row is kept. */
int mg_rollout_hdqn(const mg_params* params, const mg_state* state, const mg_traj* traj,
                    const mg_hdqn_traj* htraj, const mg_stats* stats, int8_t* goal, int8_t* goal_op,
                    double* ext_acc, int64_t n,
                    int64_t env_offset, uint64_t seed, uint64_t first_step, int32_t num_steps,
                    const void* meta_net, int32_t num_goals, const void* lower_net, int32_t reset_goal,
                    uint64_t greedy_threshold, int32_t opponent_mode, const void* opp_meta_net,
                    const void* opp_lower_net, float* ring_rows,
                    uint64_t* ring_counter, int64_t ring_capacity, uint32_t flags, void* stream);

/* status[i] = goal_status on (dx1[i], v2[i]) in fp64 (ABI 17): 0 if dx1 < -0.5 v2, 1 if dx1 < 0.5 v2,
 * else 2 -- replaces hdqn.py's goal_status (scripts/hdqn.py:223-236, dx1 = state[0], v2 = state[9]),
 * the same device function mg_rollout_hdqn evaluates on each step's fp64 x2 - x1 and v2 for the
 * intrinsic reward (:314) and the inner-loop break (:322). Device pointers, stream-ordered. */
int mg_goal_status(const double* dx1, const double* v2, int8_t* status, int64_t n, void* stream);

/* ---- replay memory (scripts/main.py:91-92, :115-119, :130-135) --------------------------------
 * rows: [capacity, row_floats] fp32 device buffer, row = [s(10), a, r, s'(10)] like
 * np.hstack((state, [action, reward], next_state)) (row_floats 22), or the goal-augmented
 * [goal, s(10), a, r, next_goal, s'(10)] of hdqn.py's lower memory (row_floats 24, tr->goal set);
 * counter: one device uint64, the reference's memory_counter.
 * mg_replay_store appends the transitions of *tr in (t, i) order -- the order in which
 * stepping env 0..n-1 at each step and calling store_transition would append them -- at
 * slot (memory_counter + k) % capacity, skipping those whose won bit is set when
 * skip_ego_won != 0 (main.py:209 `if env.winner is not 1`; hdqn.py:316 stores every one), and
 * adds the number appended to *counter. When more than capacity transitions are appended only
 * the newest capacity are written, as sequential stores would leave them. scratch: a device
 * buffer of at least mg_replay_scratch_bytes(n, num_steps) bytes, 8-byte aligned, any contents;
 * one scratch buffer per stream. Three launches, stream-ordered, no host synchronisation. */
size_t mg_replay_scratch_bytes(int64_t n, int32_t num_steps);
int mg_replay_store(float* rows, uint64_t* counter, int64_t capacity, int32_t row_floats,
                    const mg_transitions* tr, int64_t n, int32_t num_steps, int32_t skip_ego_won,
                    void* scratch, size_t scratch_bytes, void* stream);

/* out[batch, row_floats] = rows[idx[b]], idx[b] = floor(u0 * M / 2^32) with u = Philox4x32-10(key = seed,
 * counter = (b, draw)) and M = capacity (np.random.choice(MEMORY_CAPACITY, BATCH_SIZE),
 * main.py:130 -- the reference learns only once the memory is full) or, when filled_only != 0,
 * M = min(*counter, capacity) (at least 1). idx_out[batch] (int64, may be NULL) gets the slots. */
int mg_replay_sample(const float* rows, const uint64_t* counter, int64_t capacity,
                     int32_t row_floats, uint64_t seed, uint64_t draw, int32_t filled_only,
                     float* out, int64_t* idx_out, int64_t batch, void* stream);

/* (ABI 20) *totals = the n records summed on the device, in a fixed order so the fp64 sums are
 * reproducible bit for bit: blocks of 1,024 records, thread t of 256 adding records t, t + 256,
 * t + 512, t + 768 of its block in that order onto -0.0, the 256 values folded in halves
 * (v[t] += v[t + o] for o = 128, 64, ..., 1); then the block partials the same way (thread t adding
 * partials t, t + 256, ... in order, then the fold). Counts are exact. scratch: device buffer of at
 * least mg_stats_reduce_scratch_bytes(n) bytes (16-byte aligned); rec 16-byte aligned, totals (a
 * device mg_stats_totals) 8-byte aligned. Two launches, stream-ordered; n == 0 gives zero counts
 * and -0.0 sums. */
size_t mg_stats_reduce_scratch_bytes(int64_t n);
int mg_stats_reduce(const mg_episode_stats* rec, int64_t n, mg_stats_totals* totals, void* scratch,
                    size_t scratch_bytes, void* stream);

/* Resets the envs whose mask byte is non-zero (mask == NULL: all n) and writes their reset
 * observation to out->obs / out->rec64 when given. Replaces MergeEnv.reset (merging_env.py:208-230). */
int mg_reset(const mg_params* params, const mg_state* state, const uint8_t* mask,
             const mg_outputs* out, int64_t n, void* stream);

/* Observation and collision test of the current state, no state change: out->obs /
 * out->rec64 (obs only) and out->coll. Replaces MergeEnv.observe (merging_env.py:118-132)
 * and MergeEnv.is_collided (:198-206). */
int mg_observe(const mg_params* params, const mg_state* state, const mg_outputs* out, int64_t n,
               void* stream);

/* ---- host (CPU) path, ABI 20 ---------------------------------------------------------------------
 * The same step, reset and observation functions the kernels run, compiled for the host and applied
 * to HOST pointers, synchronously, one env after another: every output and condition is exactly
 * mg_step's / mg_reset's / mg_observe's (done_mask / won_mask words per 64 envs included), and the
 * doubles are the kernel's bit for bit (the host build has no contraction either; sin / cos for
 * |theta| >= 1/16, off every live-episode state, are glibc's there). For one env at the scripts'
 * pace (merging_env.py:138-230 called per step, scripts/human_player.py:112-187) a step costs
 * ~1 us here against a kernel launch plus a stream synchronisation on the GPU; batches belong on
 * the device (mg_step and the rollout kernels). */
int mg_host_step(const mg_params* params, const mg_state* state, const int8_t* a1, const int8_t* a2,
                 const mg_outputs* out, const mg_stats* stats, int64_t n, uint32_t flags);
int mg_host_reset(const mg_params* params, const mg_state* state, const uint8_t* mask,
                  const mg_outputs* out, int64_t n);
int mg_host_observe(const mg_params* params, const mg_state* state, const mg_outputs* out, int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* MERGING_HIP_H_ */
