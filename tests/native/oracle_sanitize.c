/* Host sanitizer driver for the C oracle (test infrastructure): built with
 * -fsanitize=address,undefined together with oracle/merge_oracle.c by tests/test_sanitizers.py.
 * Steps a batch through every entry point with valid, None and invalid actions, autoreset on
 * and off, every optional output present or NULL; any sanitizer report aborts the run. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct oracle_env { /* oracle/merge_oracle.c */
  double pos1, vel1, acc1, pos2, vel2, acc2, time_stamp, r1_acc, r2_acc, ep_reward_main;
  int32_t winner, done, steps, pad_;
} oracle_env;

void oracle_reset_batch(oracle_env* envs, int64_t n, double* obs);
int32_t oracle_step_batch(oracle_env* envs, int64_t n, const int8_t* a1, const int8_t* a2, int32_t autoreset,
                          double* obs, double* rew, uint8_t* done, uint8_t* coll, double* final_obs,
                          double* ret_sum, uint32_t* counts, uint32_t* status, int32_t unused);
int64_t oracle_rollout_random(oracle_env* envs, int64_t n, int64_t steps, uint64_t seed, uint64_t first_step,
                              int32_t opp_random, int64_t env_offset, double* ret_sum, uint32_t* counts);
void oracle_philox_batch(int64_t n, int64_t env_offset, uint64_t seed, uint64_t step, uint32_t* out);
void oracle_random_actions(int64_t n, int64_t env_offset, uint64_t seed, uint64_t step, int32_t opp_random,
                           int8_t* a1, int8_t* a2);

int main(void) {
  enum { N = 257, STEPS = 3000 };
  oracle_env* envs = calloc(N, sizeof(oracle_env));
  double* obs = malloc(sizeof(double) * N * 10);
  double* fobs = malloc(sizeof(double) * N * 10);
  double* rew = malloc(sizeof(double) * N * 2);
  double* ret_sum = calloc(N * 3, sizeof(double)); /* [N,3] */
  uint32_t* counts = calloc(N * 6, sizeof(uint32_t)); /* [N,6] */
  uint32_t* status = malloc(sizeof(uint32_t) * N);
  uint32_t* u = malloc(sizeof(uint32_t) * N * 4);
  uint8_t *done = malloc(N), *coll = malloc(N);
  int8_t *a1 = malloc(N), *a2 = malloc(N);
  int64_t errs = 0;
  oracle_reset_batch(envs, N, obs);
  for (int k = 0; k < STEPS; ++k) {
    oracle_random_actions(N, 0, 7, (uint64_t)k, 1, a1, a2);
    if (k % 97 == 0) { a1[k % N] = 7; a2[(k + 1) % N] = -3; } /* the reference's KeyError path */
    if (k % 5 == 0) a2[k % N] = -1;                              /* None: the L0 opponent */
    const int full = k % 3 != 0;
    errs += oracle_step_batch(envs, N, a1, k % 11 == 0 ? NULL : a2, k < 2000, full ? obs : NULL,
                              full ? rew : NULL, done, full ? coll : NULL, full ? fobs : NULL,
                              full ? ret_sum : NULL, full ? counts : NULL, full ? status : NULL, 0) != 0;
  }
  errs += 0 * oracle_rollout_random(envs, N, 64, 9, 5000, 1, 3, ret_sum, counts);
  oracle_philox_batch(N, 11, 3, 99, u);
  printf("oracle sanitizer run ok: %d envs x %d steps, %lld steps with invalid actions\n", N, STEPS,
         (long long)errs);
  free(envs); free(obs); free(fobs); free(rew); free(ret_sum); free(counts); free(status); free(u);
  free(done); free(coll); free(a1); free(a2);
  return errs > 0 ? 0 : 1; /* the invalid actions must have been reported */
}
