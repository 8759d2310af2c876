// merging_hip.hip — batched MergingEnv step for MI355X (gfx950, CDNA4).
//
// One thread owns one env. The env batch lives in HBM as a struct of arrays
// (include/merging_hip.h: mg_state); a step streams every array once in and once out,
// so the kernel is bound by HBM bandwidth, not by arithmetic (no contraction -> no MFMA).
//
// Reference being replaced (all paths relative to YikangZhang1641/merging-gym):
//   MergeEnv.step            merging_gym/envs/merging_env.py:138-195
//   MergeEnv.action_to_acc   merging_env.py:134-136  -> scripts/helper.py:152-191 mpc_1d
//   MergeEnv.observe         merging_env.py:118-132  -> lon2coord :48-58
//   MergeEnv.is_collided     merging_env.py:198-206  -> corners :232-239 (pygame Rect / Vector2,
//                                                        shapely Polygon.intersects)
//   MergeEnv.reset           merging_env.py:208-230
//
// Numerics: fp64 throughout, IEEE add/mul/div without contraction (the file is compiled
// with -ffp-contract=off and the pragma below), so positions, speeds, arrival tests and
// rewards are the same doubles the reference's Python floats hold (mpc_1d's first control
// carries the QP solver's own rounding, see mpc_acc). sin/cos: for |theta| < 1/16 (every
// live-episode state) a degree-9/10 Taylor polynomial in fma form, identical to glibc's
// sin/cos in 99.98 % of 2e7 samples and otherwise 1 ulp off; larger angles use the device
// math library (<= 1 ulp). Every other operation is correctly rounded.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "merging_hip.h"

#pragma clang fp contract(off)

namespace {

// One build, no compile-time variants: every alternative measured against the shipped choice
// (profiles/r01, profiles/r02/ab) was removed from the product source once it lost.
constexpr int kBlock = 256;  // 4 waves of 64 (128 and 512 measured within 0.8 %)
constexpr int kObs = MG_OBS_DIM;

// The step's functions compile for the host as well: the CPU single-env path (mg_host_step,
// BASELINE config 1, scripts/human_player.py's 20 Hz loop on a machine without a GPU) runs this
// same code. The host side is built with the same -ffp-contract=off, and fma / fabs / sqrt are
// correctly rounded there too, so host and device give the same doubles; only the cold sin/cos
// branch (|theta| >= 1/16, off every live-episode state) uses glibc on the host.
#define MG_HD __host__ __device__ __forceinline__
#define MG_STR_(x) #x
#define MG_STR(x) MG_STR_(x)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// Store of a per-step output (observation, reward, flags, actions): written once, never
// re-read by the step, so optionally non-temporal. The env state is stored normally: the
// next step reads it back (write-through or non-temporal state stores measured 0 to +4 %).
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

template <class T>
MG_HD void st_state(T* p, T v) {
  *p = v;
}

// Action codes after host/device decoding: 0..4 valid, -1 None (opponent only), anything
// else is the reference's KeyError.
MG_HD bool valid_action(int a) { return a >= 0 && a < MG_NUM_ACTIONS; }

// x / d for a divisor fixed per launch, correctly rounded: q = x * (1/d), then Markstein's
// FMA correction. With inv = RN(1/d) this returns RN(x / d) for d = 3 and d = 30000 (the
// only divisors used; 0 mismatches in 8e8 random tests, incl. random exponents,
// tests/test_division.py) at 3 instructions instead of the ~10 of a general fp64 division.
MG_HD double div_const(double x, double d, double inv) {
  const double q = x * inv;
  const double r = fma(-q, d, x);
  return fma(r, inv, q);
}

// sin and cos of the double theta. For |theta| < 1/16 -- pos in [-875, 2875], which covers
// every state of a live episode (pos 50..~1000) -- a degree-9 / degree-10 Taylor polynomial
// in fma form: the correction terms are < 7e-4 of the result, so the one rounding of the
// final fma dominates and the result agrees with libm's sin/cos to <= 1 ulp (identical in
// 99.98 % of 2e7 samples vs glibc). Larger |theta| takes the device library's sincos.
// The device library's sincos for |t| >= 1/16 (only reached off the live-episode range, e.g.
// stepping far past done). Kept out of line: inlined, the compiler hoists its polynomial
// constants into VGPRs for the whole step loop of the T-step kernels, which then spill. Its
// results come back by value (round 4): through pointers they were private-memory loads in the
// caller, and the wait for those at the join after the branch -- one in-order counter for vector
// loads and stores on gfx950 -- also waited for every store the wave had in flight, on the common
// path too. Config 5 -1.5 to -3 % per step, the rollout and h-DQN within noise (profiles/r04/ab/
// r04z_*, and r04ab_*: the rollout in both orders, and by-value in the lockstep path only, which tied).
__device__ __attribute__((noinline, unused)) double2 sincos_cold(double t) {
  double s, c;
  sincos(t, &s, &c);
  return make_double2(s, c);
}

// the polynomial branch (|t| < 1/16)
MG_HD void sincos_poly(double t, double& s, double& c) {
  const double t2 = t * t;
  const double ps = fma(t2, fma(t2, fma(t2, 2.7557319223985893e-06, -1.9841269841269841e-04),
                                8.3333333333333332e-03),
                        -1.6666666666666666e-01);
  s = fma(t * t2, ps, t);
  const double pc =
      fma(t2, fma(t2, fma(t2, fma(t2, -2.7557319223985888e-07, 2.4801587301587302e-05),
                          -1.3888888888888889e-03),
                  4.1666666666666664e-02),
          -0.5);
  c = fma(t2, pc, 1.0);
}

MG_HD void arc_sincos(double t, double& s, double& c) {
  if (fabs(t) < 0.0625) {
    sincos_poly(t, s, c);
    return;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const double2 sc = sincos_cold(t);
  s = sc.x;
  c = sc.y;
#else
  s = std::sin(t);
  c = std::cos(t);
#endif
}

// arc_sincos of M angles: when every one is in the polynomial's range (the usual case) the M
// polynomials form one straight-line block the scheduler can interleave; otherwise each angle
// takes arc_sincos's own branch. Same results as M arc_sincos calls.
template <int M>
__device__ __forceinline__ void arc_sincos_n(const double (&t)[M], double (&s)[M], double (&c)[M]) {
  bool fast = true;
#pragma unroll
  for (int k = 0; k < M; ++k) fast = fast && fabs(t[k]) < 0.0625;
  if (fast) {
#pragma unroll
    for (int k = 0; k < M; ++k) sincos_poly(t[k], s[k], c[k]);
    return;
  }
#pragma unroll
  for (int k = 0; k < M; ++k) arc_sincos(t[k], s[k], c[k]);
}

// lon2coord (merging_env.py:48-58): position along the arc -> (x longitudinal, y lateral).
// The ego rides the arc on +y, the opponent its mirror image on -y. Split in three so the
// lockstep step can batch the sin/cos of several cars.
MG_HD double arc_angle(const mg_params& P, double lon) {
  return P.angle0 - div_const(lon, P.R, P.inv_R);
}

MG_HD void arc_xy(const mg_params& P, double s, double c, bool ego, double& x,
                                       double& y) {
  x = P.R * s;
  const double d = P.R - P.R * c;
  const double half_w = P.W * 0.5;  // W/2 = 150.0 exactly
  y = ego ? (half_w + d) : (half_w - d);
}

MG_HD void lon2coord(const mg_params& P, double lon, bool ego, double& x,
                                          double& y) {
  double s, c;
  arc_sincos(arc_angle(P, lon), s, c);
  arc_xy(P, s, c, ego, x, y);
}

// corners (merging_env.py:232-239) is called as corners(agent, y=x, x=y, 0) (:201-202), so
// the pygame Rect is centred at (lateral, longitudinal) with w = VEHICLE_W (lateral) and
// h = VEHICLE_H (longitudinal) (surfaces :97-98). pygame converts a float centre with a C
// (int) cast, i.e. truncation toward zero, then sets x = cx - w/2, y = cy - h/2. Each corner
// is ((double)corner - pivot) + pivot in fp64 (Vector2 difference, rotate(0) = identity,
// 1.0 * v, + pivot), which is not always the integer corner (no Sterbenz near 0).
struct Box {
  double l, r, t, b;  // lateral [l, r], longitudinal [t, b]
};

MG_HD Box vehicle_box(const mg_params& P, double lat, double lon) {
  const int rx = static_cast<int>(lat) - P.veh_w / 2;
  const int ry = static_cast<int>(lon) - P.veh_h / 2;
  Box bx;
  bx.l = (static_cast<double>(rx) - lat) + lat;
  bx.r = (static_cast<double>(rx + P.veh_w) - lat) + lat;
  bx.t = (static_cast<double>(ry) - lon) + lon;
  bx.b = (static_cast<double>(ry + P.veh_h) - lon) + lon;
  return bx;
}

// shapely Polygon.intersects on two axis-aligned rectangles: the closed boxes share a point.
MG_HD bool boxes_intersect(const Box& a, const Box& b) {
  return a.l <= b.r && b.l <= a.r && a.t <= b.b && b.t <= a.b;
}

// is_collided (:198-206) of cars at (lateral y, longitudinal x): boxes_intersect(vehicle_box(y1, x1),
// vehicle_box(y2, x2)) with the lateral edges as integers where that is exact. For y >= 8 the corner
// k = trunc(y) - w/2 (or + w/2) lies within [y/2, 2y], so k - y is exact (Sterbenz) and (k - y) + y is
// k itself: the fp64 lateral edges are the integer ones and their comparison is an integer one. Every
// lateral coordinate of a live episode is 150 +- d with d <= 59 (|theta| < 1/16); the opponent's mirror
// arc reaches y < 8 only far past the end of an episode, where the fp64 form stays. Same result as
// the fp64 test for every input (tests/test_host_step.py drives both on the host).
MG_HD bool vehicles_collide(const mg_params& P, double y1, double x1, double y2, double x2) {
  if (y1 >= 8.0 && y2 >= 8.0) {
    const int l1 = static_cast<int>(y1) - P.veh_w / 2, l2 = static_cast<int>(y2) - P.veh_w / 2;
    if (l1 > l2 + P.veh_w || l2 > l1 + P.veh_w) return false;
    const int t1 = static_cast<int>(x1) - P.veh_h / 2, t2 = static_cast<int>(x2) - P.veh_h / 2;
    const double a_t = (static_cast<double>(t1) - x1) + x1, a_b = (static_cast<double>(t1 + P.veh_h) - x1) + x1;
    const double b_t = (static_cast<double>(t2) - x2) + x2, b_b = (static_cast<double>(t2 + P.veh_h) - x2) + x2;
    return a_t <= b_b && b_t <= a_b;
  }
  return boxes_intersect(vehicle_box(P, y1, x1), vehicle_box(P, y2, x2));
}

// observe (merging_env.py:118-132): computed in fp64, stored as OT (fp64 for the single-env
// record; fp32 -- the one rounding every fp32 output gets -- for the batched kernels)
template <class OT>
MG_HD void observe(const mg_params& P, double p1, double v1, double p2,
                                        double v2, double x1, double y1, double x2, double y2,
                                        OT (&o)[kObs]) {
  o[0] = static_cast<OT>(x2 - x1);
  o[1] = static_cast<OT>(y2 - y1);
  o[2] = static_cast<OT>(v2 - v1);
  o[3] = static_cast<OT>(P.end_point - p1);
  o[4] = static_cast<OT>(v1);
  o[5] = static_cast<OT>(x1 - x2);
  o[6] = static_cast<OT>(y1 - y2);
  o[7] = static_cast<OT>(v1 - v2);
  o[8] = static_cast<OT>(P.end_point - p2);
  o[9] = static_cast<OT>(v2);
}

template <class OT>
MG_HD void reset_obs(const mg_params& P, OT (&o)[kObs], double* dx1 = nullptr) {
  double x1, y1, x2, y2;
  lon2coord(P, P.start_point, true, x1, y1);
  lon2coord(P, P.start_point, false, x2, y2);
  observe(P, P.start_point, P.start_vel, P.start_point, P.start_vel, x1, y1, x2, y2, o);
  if (dx1) *dx1 = x2 - x1;
}

// The reset observation (merging_env.py:208-230 then observe): the same ten fp32 values and fp64
// x2 - x1 for every env, so each launch computes it once on the host (the same MG_HD functions, the
// same doubles) and the kernels copy it from the launch arguments (scalar loads) where autoreset
// fires, instead of two sin / cos and the observation in the divergent finishing branch.
struct Reset0 {
  float o[kObs];
  double dx1;
};

MG_HD Reset0 reset0(const mg_params& P) {
  Reset0 z;
  reset_obs(P, z.o, &z.dx1);
  return z;
}

// goal_status (scripts/hdqn.py:223-236) on the reference's fp64 values: dx1 = state[0] = x2 - x1,
// v2 = state[9] (an int 0 after max(0, ...) compares as 0.0). 0: dx1 < -v2/2, 1: dx1 < v2/2, else 2.
MG_HD int goal_status(double dx1, double v2) {
  return dx1 < -0.5 * v2 ? 0 : (dx1 < 0.5 * v2 ? 1 : 2);
}

// Philox4x32-10 (Salmon et al., SC'11 "Parallel random numbers: as easy as 1, 2, 3").
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}

// floor(5 u / 2^32): uniform over {0..4} up to a 5/2^32 bias.
__device__ __forceinline__ int action_from_u32(uint32_t u) {
  return static_cast<int>((static_cast<uint64_t>(u) * MG_NUM_ACTIONS) >> 32);
}

enum ActMode { kActArrays = 0, kActPhilox = 1 };

// One env's state, held in registers for the duration of a launch.
struct Env {
  double p1, v1, p2, v2, ret1, ret2;
  uint32_t steps, winner;
  bool done;
};

MG_HD Env load_env(const mg_state& S, int64_t i) {
  Env e;
  e.p1 = S.p1[i];
  e.v1 = S.v1[i];
  e.p2 = S.p2[i];
  e.v2 = S.v2[i];
  e.ret1 = S.ret1[i];
  e.ret2 = S.ret2[i];
  const uint32_t tf = S.tf[i];
  e.steps = tf & MG_TF_STEPS_MASK;
  e.winner = (tf & MG_TF_WINNER_MASK) >> MG_TF_WINNER_SHIFT;
  e.done = (tf & MG_TF_DONE) != 0;
  return e;
}

MG_HD uint32_t pack_tf(const Env& e) {
  return e.steps | (e.winner << MG_TF_WINNER_SHIFT) | (e.done ? MG_TF_DONE : 0u);
}

MG_HD void store_env(const mg_state& S, int64_t i, const Env& e) {
  st_state(S.p1 + i, e.p1);
  st_state(S.v1 + i, e.v1);
  st_state(S.p2 + i, e.p2);
  st_state(S.v2 + i, e.v2);
  st_state(S.ret1 + i, e.ret1);
  st_state(S.ret2 + i, e.ret2);
  st_state(S.tf + i, static_cast<uint16_t>(pack_tf(e)));
}

// What one step returns besides the new state.
// The observation a step hands back, held as fp32: every batched output is fp32, and fp32
// here frees 10 VGPRs (66 -> fewer in the one-step kernel). The single-env record, which returns
// the reference's fp64 floats, recomputes its observation in fp64 from the state.
typedef float obs_t;

struct StepOut {
  obs_t o[kObs];  // observation (the reset observation once autoreset has fired)
  double r1, r2, acc1, acc2;
  double dx1;     // x2 - x1 of o in fp64 (hdqn.py goal_status's dx1; the reset one after autoreset)
  double ret_pre; // r1_accumulate before this step (read where first1)
  bool done, coll, r1_int, r2_int, v1_int, v2_int;
  bool first1;    // the ego arrived first on this step (winner None -> 1, merging_env.py:164-166)
  bool win_pre;   // main.py:225's END_POINT - p2 > END_POINT - p1 on the state this step acted on
  int bad;  // 1: action1 invalid, 2: action2 invalid (the reference's KeyError)
};

// The random-policy action stream: step k of global env gi takes word (k div 2) mod 4 of
// u = Philox4x32-10(counter (gi, k div 8), key seed) -- one call covers eight steps, two draws per
// 32-bit word, so a T-step rollout pays an eighth of a call's 40 multiplies per env-step (one call
// per step had been a third of the rollout kernel's VALU). A draw of m outcomes from word w is
// floor(m w / 2^32); an odd step draws from w' = m w mod 2^32 instead, the remainder of the first
// draw (m is odd, so w -> w' is a bijection of the 32-bit words and w' is again uniform; the two
// draws of one word are independent up to an m^2 / 2^32 bias). With both players random m = 25 and
// x = draw is the action pair, a1 = x div 5, a2 = x mod 5; with the None opponent m = 5, a1 = draw.
__device__ __forceinline__ uint4 philox_block(uint64_t gi, uint64_t block, uint64_t seed,
                                              bool opaque_key = false) {
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  // opaque_key: a uniform key the compiler cannot hoist. In a multi-step loop the 20 round keys
  // are then scalar adds at each use instead of loop invariants spilled into VGPR lanes (one
  // v_readlane, a vector instruction, per round): -2 % per rollout step (A/B).
  if (opaque_key) asm volatile("" : "+s"(k0), "+s"(k1));
  return philox4x32_10(make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32),
                                  static_cast<uint32_t>(block), static_cast<uint32_t>(block >> 32)),
                       k0, k1);
}

constexpr int kStepsPerPhilox = 8;  // steps one Philox4x32-10 call feeds: 4 words x 2 draws

__device__ __forceinline__ void actions_from_block(const uint4& u, uint64_t step, int opp_random, int& a1,
                                                   int& a2) {
  // word (step div 2) & 3 by a 64-bit select and shift on values: no indexed private array, no branch
  const uint64_t lo = (static_cast<uint64_t>(u.y) << 32) | u.x, hi = (static_cast<uint64_t>(u.w) << 32) | u.z;
  const uint32_t m = opp_random ? 25u : static_cast<uint32_t>(MG_NUM_ACTIONS);
  uint32_t w = static_cast<uint32_t>(((step & 4) ? hi : lo) >> (32 * ((step >> 1) & 1)));
  if (step & 1) w *= m;  // the second draw of the word
  const uint32_t x = static_cast<uint32_t>((static_cast<uint64_t>(w) * m) >> 32);
  const int b1 = static_cast<int>((x * 13u) >> 6);  // x div 5 for x < 25
  a1 = opp_random ? b1 : static_cast<int>(x);
  a2 = opp_random ? static_cast<int>(x) - 5 * b1 : MG_ACTION_NONE;
}

__device__ __forceinline__ void draw_actions(uint64_t gi, uint64_t step, uint64_t seed, int opp_random,
                                             int& a1, int& a2) {
  actions_from_block(philox_block(gi, step / kStepsPerPhilox, seed), step, opp_random, a1, a2);
}

// time_stamp += dT; done if time_stamp > 500 (:141-143). The fp64 clock first exceeds 500
// on step 2501; an integer count reproduces that exactly.
MG_HD void env_clock(const mg_params& P, Env& e) {
  e.steps = e.steps < MG_TF_STEPS_MASK ? e.steps + 1 : e.steps;
  if (static_cast<int32_t>(e.steps) >= P.timeout_steps) e.done = true;
}

// mpc_1d (helper.py:152-191): min u'(D'D + 0.01 I)u s.t. A[1] u = b, b = vt - v0 (only the
// velocity row of the constraint reaches solve_qp, :172-173, :182). quadprog's dual active-set
// method starts at the unconstrained minimiser u = 0 and adds the one equality in a single step,
// u = (b / z'n) z with z = J J'n, J = R^-1; action() = u[0]. z'n and z[0] are per-launch
// constants (mg_params.qp_nz / qp_z0, computed by mg_params_default in qpgen2's operation order),
// so this is two correctly rounded operations with the solver's own rounding; a residual |b| below
// qpgen2's vsmall counts as already satisfied and leaves the unconstrained minimiser u = -0.0 (dposl
// of a = -q, q = 0). (Mathematically u0 = b / t, since
// D.1 = 0; evaluating that closed form instead moves u0 by an ulp in most steps.)
MG_HD double mpc_acc_speed(const mg_params& P, double speed, double v) {
  const double b = speed - v;
  const double u = div_const(b, P.qp_nz, P.qp_inv_nz) * P.qp_z0;
  return fabs(b) < P.qp_vsmall ? -0.0 : u;  // dposl's -0.0 (a = -q = -0.0): nothing violated
}

MG_HD double mpc_acc(const mg_params& P, int a, double v) {
  return mpc_acc_speed(P, P.action_speed[a], v);
}

// action_dict[a] (merging_env.py:101) or 0.0 where a is not in it (the value is then unused)
MG_HD double action_speed_or0(const mg_params& P, int a) {
  return valid_action(a) ? P.action_speed[a] : 0.0;
}

// v = max(0, v + acc*dT) (an int 0 when the max picks 0), p += v*dT  (:149-150, :153-154)
MG_HD void move_car(const mg_params& P, double acc, double& p, double& v,
                                         bool& v_int) {
  const double nv = v + acc * P.dT;
  v_int = !(nv > 0.0);
  v = v_int ? 0.0 : nv;
  p = p + v * P.dT;
}

MG_HD void score_step(const mg_params& P, Env& e, double x1, double y1,
                                           double x2, double y2, StepOut& r, bool frozen = false);

// main.py:225's win test, state[8] > state[3] = END_POINT - p2 > END_POINT - p1, on the state a step
// acts on, evaluated before the move: left to the compiler it sinks into the rare finishing branch
// and keeps the pre-step positions live across the step (66 instead of 61 VGPRs in the step
// kernel: 7 waves per SIMD, a third round of blocks at 2^20 envs).
MG_HD bool win_test_early(const mg_params& P, const Env& e) {
  int w = (P.end_point - e.p2) > (P.end_point - e.p1) ? 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(w));
#endif
  return w != 0;
}

// MergeEnv.step (merging_env.py:138-195) for one env held in registers. CHECKED = false: the
// caller guarantees a1 in 0..4 and a2 in -1..4 (device-drawn actions), so the KeyError path and
// its zeroed outputs are not compiled in.
// sp1 / sp2: action_dict[a1] / [a2], looked up by the caller (action_speed_or0), so it can issue
// those loads before the state loads (the step kernel; env_step below looks them up itself)
template <bool CHECKED = true>
MG_HD void env_step_sp(const mg_params& P, Env& e, int a1, int a2, double sp1, double sp2,
                                            StepOut& r) {
  r.win_pre = win_test_early(P, e);
  r.first1 = false;
  r.dx1 = 0.0;
  env_clock(P, e);
  const bool bad1 = CHECKED && !valid_action(a1);
  const bool bad2 = CHECKED && !(a2 == MG_ACTION_NONE || valid_action(a2));
  r.bad = (bad1 ? 1 : 0) | (bad2 ? 2 : 0);
  r.acc1 = r.acc2 = 0.0;
  r.v1_int = r.v2_int = false;
  r.done = r.coll = r.r1_int = r.r2_int = false;
  r.r1 = r.r2 = 0.0;
  if (!bad1) {
    r.acc1 = mpc_acc_speed(P, sp1, e.v1);
    move_car(P, r.acc1, e.p1, e.v1, r.v1_int);
  }
  if (r.bad) {  // the reference raises KeyError at action_dict[...] after advancing this far
#pragma unroll
    for (int k = 0; k < kObs; ++k) r.o[k] = 0.0;
    return;
  }
  // action2 None -> acc 0 (:152): the "L0" constant-speed opponent
  if (a2 != MG_ACTION_NONE) r.acc2 = mpc_acc_speed(P, sp2, e.v2);
  move_car(P, r.acc2, e.p2, e.v2, r.v2_int);

  double x1, y1, x2, y2;
  lon2coord(P, e.p1, true, x1, y1);
  lon2coord(P, e.p2, false, x2, y2);
  score_step(P, e, x1, y1, x2, y2, r);
}

template <bool CHECKED = true>
MG_HD void env_step(const mg_params& P, Env& e, int a1, int a2, StepOut& r) {
  env_step_sp<CHECKED>(P, e, a1, a2, action_speed_or0(P, a1), action_speed_or0(P, a2), r);
}

// N envs stepped statement by statement, so their independent fp64 chains interleave in one
// instruction stream. Identical results to N env_step calls, invalid actions included: those
// are computed with a stand-in action and their effects dropped by selects (the ego keeps its
// move unless action1 is bad; nothing after the moves happens, as in env_step's early return).
template <int N, bool CHECKED = true>
__device__ __forceinline__ void env_step_lockstep(const mg_params& P, Env (&e)[N], const int (&a1)[N],
                                                  const int (&a2)[N], StepOut (&r)[N]) {
  double ang[2 * N], sn[2 * N], cs[2 * N];
  bool bad[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool bad1 = CHECKED && !valid_action(a1[j]);
    const bool none2 = a2[j] == MG_ACTION_NONE;
    const bool bad2 = CHECKED && !(none2 || valid_action(a2[j]));
    bad[j] = bad1 || bad2;
    r[j].bad = (bad1 ? 1 : 0) | (bad2 ? 2 : 0);
    r[j].r1_int = r[j].r2_int = false;
    r[j].win_pre = win_test_early(P, e[j]);
    r[j].first1 = false;
    env_clock(P, e[j]);
    const double acc1 = mpc_acc(P, bad1 ? 0 : a1[j], e[j].v1);
    r[j].acc1 = bad1 ? 0.0 : acc1;
    double p = e[j].p1, v = e[j].v1;
    bool vi;
    move_car(P, r[j].acc1, p, v, vi);
    e[j].p1 = bad1 ? e[j].p1 : p;
    e[j].v1 = bad1 ? e[j].v1 : v;
    r[j].v1_int = !bad1 && vi;
    const double acc2 = mpc_acc(P, (none2 || bad2) ? 0 : a2[j], e[j].v2);
    r[j].acc2 = (none2 || bad[j]) ? 0.0 : acc2;
    p = e[j].p2;
    v = e[j].v2;
    move_car(P, r[j].acc2, p, v, vi);
    e[j].p2 = bad[j] ? e[j].p2 : p;
    e[j].v2 = bad[j] ? e[j].v2 : v;
    r[j].v2_int = !bad[j] && vi;
    ang[2 * j] = arc_angle(P, e[j].p1);
    ang[2 * j + 1] = arc_angle(P, e[j].p2);
  }
  arc_sincos_n<2 * N>(ang, sn, cs);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double x1, y1, x2, y2;
    arc_xy(P, sn[2 * j], cs[2 * j], true, x1, y1);
    arc_xy(P, sn[2 * j + 1], cs[2 * j + 1], false, x2, y2);
    score_step(P, e[j], x1, y1, x2, y2, r[j], bad[j]);
  }
}

// The rest of a step once both cars have moved (merging_env.py:156-192): observation, rewards,
// arrival / winner, collision, returns. r.r1_int / r.r2_int must be false on entry. frozen: an
// invalid action -- the step stops before any of this (observation and rewards 0, no state
// change), as env_step's early return.
MG_HD void score_step(const mg_params& P, Env& e, double x1, double y1,
                                           double x2, double y2, StepOut& r, bool frozen) {
  observe(P, e.p1, e.v1, e.p2, e.v2, x1, y1, x2, y2, r.o);
  r.dx1 = x2 - x1;
  r.ret_pre = e.ret1;
  if (frozen) {
#pragma unroll
    for (int k = 0; k < kObs; ++k) r.o[k] = 0.0;
  }

  // rewards (:158-159): -time_penalty - vel_penalty * |v - 20|
  double r1 = (0.0 - P.time_penalty) - P.vel_penalty * fabs(e.v1 - P.vel_ref);
  double r2 = (0.0 - P.time_penalty) - P.vel_penalty * fabs(e.v2 - P.vel_ref);

  // arrival / winner state machine (:163-181); ego strict '>', opponent '>='
  if (!frozen && e.p1 > P.end_point) {
    if (e.winner == 0) {
      e.winner = 1;
      r1 += P.r_first;
      r.first1 = true;
    } else if (e.winner == 1) {
      r1 = 0.0;
      r.r1_int = true;
    } else {
      r1 += P.r_second;
      e.done = true;
    }
  }
  if (!frozen && e.p2 >= P.end_point) {
    if (e.winner == 0) {
      e.winner = 2;
      r2 += P.r_first;
    } else if (e.winner == 2) {
      r2 = 0.0;
      r.r2_int = true;
    } else {
      r2 += P.r_second;
      e.done = true;
    }
  }

  // is_collided (:183-187, :198-206)
  r.coll = !frozen && vehicles_collide(P, y1, x1, y2, x2);
  if (r.coll) {
    e.done = true;
    r1 += P.r_collision;
    r2 += P.r_collision;
  }
  if (!frozen) {
    e.ret1 += r1;  // :191-192
    e.ret2 += r2;
  }
  r.r1 = frozen ? 0.0 : r1;
  r.r2 = frozen ? 0.0 : r2;
  r.done = !frozen && e.done;
}

// Completed-episode statistics (mg_episode_stats) of one env held in registers for a multi-step
// launch: the fp64 sums and ret1_pending are loaded once and accumulated in the same order as the
// per-step read-modify-write (so bit-identical); the counts are this launch's increments, added
// to the record once at the end. A finishing lane then never waits on a global load.
// The counts are 16-bit fields of three words (a launch finishes at most num_steps <= 65535
// episodes per env, mg_rollout_random checks it): two VGPRs fewer, which keeps the rollout
// kernel within 128 VGPRs (4 waves per SIMD).
struct EpStats {
  double r1, r2, rm, pend;
  uint32_t ep_coll;   // episodes | collisions << 16
  uint32_t ego_wm;    // ego_first | win_main << 16
  uint32_t wh;        // win_hdqn
  uint32_t steps;
  bool dirty_f, dirty_c;  // the fp64 half / the counts changed
};

// the record as 4 x 16 bytes: {ret[0], ret[1]}, {ret_main, ret1_pending}, counts 0-3, counts 4-7
MG_HD double2* stats_f64(const mg_stats& St, int64_t i) {
  return reinterpret_cast<double2*>(St.rec + i);
}
MG_HD uint4* stats_u32(const mg_stats& St, int64_t i) {
  return reinterpret_cast<uint4*>(St.rec + i) + 2;
}

MG_HD void stats_load(const mg_stats& St, int64_t i, EpStats& s) {
  s.dirty_f = s.dirty_c = false;
  s.r1 = s.r2 = s.rm = s.pend = 0.0;
  s.ep_coll = s.ego_wm = s.wh = s.steps = 0u;
  if (St.rec) {
    const double2 a = stats_f64(St, i)[0], b = stats_f64(St, i)[1];
    s.r1 = a.x;
    s.r2 = a.y;
    s.rm = b.x;
    s.pend = b.y;
  }
}

MG_HD void stats_store(const mg_stats& St, int64_t i, const EpStats& s) {
  if (!St.rec) return;
  if (s.dirty_f) {
    stats_f64(St, i)[0] = make_double2(s.r1, s.r2);
    stats_f64(St, i)[1] = make_double2(s.rm, s.pend);
  }
  if (s.dirty_c) {  // once per launch: the load's latency is not on the step loop
    uint4 c = stats_u32(St, i)[0], d = stats_u32(St, i)[1];
    c.x += s.ep_coll & 0xFFFFu;
    c.y += s.ep_coll >> 16;
    c.z += s.ego_wm & 0xFFFFu;
    c.w += s.steps;
    d.x += s.ego_wm >> 16;
    d.y += s.wh;
    stats_u32(St, i)[0] = c;
    stats_u32(St, i)[1] = d;
  }
}

// The ego arrived first on a step that did not end the episode: keep r1_accumulate as it stood
// before that step -- main.py's ep_reward stops there (:209-211), since winner stays 1.
MG_HD void note_first_arrival(const mg_stats& St, int64_t i, const StepOut& r,
                                                   EpStats* sreg = nullptr) {
  if (sreg) {
    sreg->pend = r.ret_pre;
    sreg->dirty_f = true;
  } else if (St.rec) {
    reinterpret_cast<double*>(St.rec + i)[3] = r.ret_pre;  // ret1_pending
  }
}

// gym.vector autoreset after the episode was recorded: keep its terminal observation, reset the
// env (merging_env.py:208-230) and put the reset observation in r.o (r0: the launch's precomputed
// one, reset0).
MG_HD void autoreset_env(const mg_params& P, Env& e, StepOut& r, float* final_obs_row, const Reset0* r0) {
  if (final_obs_row) {
#pragma unroll
    for (int k = 0; k < kObs; ++k) final_obs_row[k] = static_cast<float>(r.o[k]);
  }
  e.p1 = e.p2 = P.start_point;
  e.v1 = e.v2 = P.start_vel;
  e.ret1 = e.ret2 = 0.0;
  e.steps = 0;
  e.winner = 0;
  e.done = false;
  if (r0) {
#pragma unroll
    for (int k = 0; k < kObs; ++k) r.o[k] = r0->o[k];
    r.dx1 = r0->dx1;
  } else {
    reset_obs(P, r.o, &r.dx1);
  }
}

// Record the finished episode, then autoreset (autoreset_env). sreg: statistics held in registers
// (the random rollout), nullptr: read-modify-write them in memory (the one-step kernels and the host
// path; the Q-net kernels use finish_episode_nowait below). The episode's statistics:
// r{1,2}_accumulate (hdqn.py's ep_reward), main.py's winner-filtered ep_reward (r1_accumulate
// before the ego-first step while winner == 1), main.py:225's win test on the state the last step
// acted on (r.win_pre) and hdqn.py:342's on the terminal state.
MG_HD void finish_episode(const mg_params& P, Env& e, StepOut& r,
                                               const mg_stats& St, float* final_obs_row,
                                               int64_t i, EpStats* sreg = nullptr, const Reset0* r0 = nullptr) {
  const bool ego_won = e.winner == 1;
  const bool win_hdqn = (P.end_point - e.p2) > (P.end_point - e.p1);
  if (sreg) {
    const double pend = r.first1 ? r.ret_pre : sreg->pend;
    sreg->r1 += e.ret1;
    sreg->r2 += e.ret2;
    sreg->rm += ego_won ? pend : e.ret1;
    sreg->ep_coll += 1u + (r.coll ? 0x10000u : 0u);
    sreg->ego_wm += (ego_won ? 1u : 0u) + (r.win_pre ? 0x10000u : 0u);
    sreg->wh += win_hdqn ? 1u : 0u;
    sreg->steps += e.steps;
    sreg->dirty_f = sreg->dirty_c = true;
  } else if (St.rec) {
    // one 64-byte record per env: a finishing env reads and writes one cache line
    double2* fp = stats_f64(St, i);
    const double2 a = fp[0], b = fp[1];
    const double pend = r.first1 ? r.ret_pre : b.y;
    fp[0] = make_double2(a.x + e.ret1, a.y + e.ret2);
    fp[1] = make_double2(b.x + (ego_won ? pend : e.ret1), b.y);
    uint4* cp = stats_u32(St, i);
    uint4 c = cp[0];
    uint2 d = reinterpret_cast<const uint2*>(cp + 1)[0];
    c.x += 1;
    c.y += r.coll ? 1u : 0u;
    c.z += ego_won ? 1u : 0u;
    c.w += e.steps;
    d.x += r.win_pre ? 1u : 0u;
    d.y += win_hdqn ? 1u : 0u;
    cp[0] = c;
    reinterpret_cast<uint2*>(cp + 1)[0] = d;
  }
  autoreset_env(P, e, r, final_obs_row, r0);
}

// After a step with statistics: the first-arrival bookkeeping, then autoreset where done.
MG_HD void after_step(const mg_params& P, Env& e, StepOut& r, const mg_stats& St,
                                           float* final_obs_row, int64_t i, bool autoreset,
                                           EpStats* sreg = nullptr, const Reset0* r0 = nullptr) {
  const bool finish = autoreset && r.done;
  if (r.first1 && !finish) note_first_arrival(St, i, r, sreg);
  if (finish) finish_episode(P, e, r, St, final_obs_row, i, sreg, r0);
}

// Episode statistics without a load on the step path (round 4), for the batched device kernels: a
// finishing env's record update is a handful of no-return atomics, so the lane never waits for its
// record (finish_episode's read-modify-write stalls the wave on a global load). The env's lane is
// the only writer of its record during a launch and atomics from one lane to one address are
// performed in issue order, so the sums are the sequential ones, bit for bit. The one value read
// back at an episode end is main.py's pending r1_accumulate (ret1_pending), and only when the ego
// arrived first on an earlier step: it is held in a register `pend`, loaded at the launch start
// for the lanes whose episode is in that state (pend_load: winner == 1, a small fraction) and set
// on the first arrival (also stored to the record then, a store without a wait).
__device__ __forceinline__ double pend_load(const mg_stats& St, int64_t i, const Env& e) {
  return St.rec && e.winner == 1 ? St.rec[i].ret1_pending : 0.0;
}

__device__ __forceinline__ void finish_episode_nowait(const mg_params& P, Env& e, StepOut& r, const mg_stats& St,
                                                      float* final_obs_row, int64_t i, double pend,
                                                      const Reset0* r0) {
  if (St.rec) {
    mg_episode_stats* rec = St.rec + i;
    const bool ego_won = e.winner == 1;
    const bool win_hdqn = (P.end_point - e.p2) > (P.end_point - e.p1);
    unsafeAtomicAdd(&rec->ret[0], e.ret1);
    unsafeAtomicAdd(&rec->ret[1], e.ret2);
    unsafeAtomicAdd(&rec->ret_main, ego_won ? (r.first1 ? r.ret_pre : pend) : e.ret1);
    atomicAdd(&rec->episodes, 1u);
    atomicAdd(&rec->steps, e.steps);
    if (r.coll) atomicAdd(&rec->collisions, 1u);
    if (ego_won) atomicAdd(&rec->ego_first, 1u);
    if (r.win_pre) atomicAdd(&rec->win_main, 1u);
    if (win_hdqn) atomicAdd(&rec->win_hdqn, 1u);
  }
  autoreset_env(P, e, r, final_obs_row, r0);
}

// after_step with the no-wait statistics; returns whether the episode finished (autoreset)
__device__ __forceinline__ bool after_step_nowait(const mg_params& P, Env& e, StepOut& r, const mg_stats& St,
                                                  float* final_obs_row, int64_t i, bool autoreset, double& pend,
                                                  const Reset0* r0) {
  const bool finish = autoreset && r.done;
  if (finish) {
    finish_episode_nowait(P, e, r, St, final_obs_row, i, pend, r0);
  } else if (r.first1) {
    pend = r.ret_pre;
    if (St.rec) St.rec[i].ret1_pending = r.ret_pre;  // note_first_arrival
  }
  return finish;
}

// The Q value a finished episode adds to its record (mg_episode_stats.q_eval), without a wait
__device__ __forceinline__ void add_q_eval_nowait(const mg_stats& St, int64_t i, double q) {
  if (St.rec) unsafeAtomicAdd(&St.rec[i].q_eval, q);
}

// Wave-scope ordering of LDS accesses between the lanes of ONE wave (no s_barrier): the LDS
// executes a wave's accesses in order; this only stops the compiler from moving them.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A wave's [rows,10] fp32 observations written through its LDS slice as contiguous 16-byte stores
// (64 rows of 40 B become 160 dwordx4 lanes instead of 640 scattered dwords): the slice holds the
// new observations afterwards, and no other wave is waited for (no block barrier).
__device__ __forceinline__ void wave_copy_rows(const float* wtile, float* dst, int nrows);

__device__ __forceinline__ void wave_store_obs(float* wtile, const obs_t (&o)[kObs], float* dst,
                                               int nrows) {
  const int lane = threadIdx.x & 63;
  float2* t2 = reinterpret_cast<float2*>(wtile + lane * kObs);
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k)
    t2[k] = make_float2(static_cast<float>(o[2 * k]), static_cast<float>(o[2 * k + 1]));
  wave_lds_sync();
  wave_copy_rows(wtile, dst, nrows);
  wave_lds_sync();
}

// wave_store_obs for N consecutive 64-row slices (slice j = r[j].o of every lane), written out
// as one run of nrows <= 64 N rows.
template <int N>
__device__ __forceinline__ void wave_store_obs_n(float* wtile, const StepOut (&r)[N], float* dst,
                                                 int nrows) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float2* t2 = reinterpret_cast<float2*>(wtile + (64 * j + lane) * kObs);
#pragma unroll
    for (int k = 0; k < kObs / 2; ++k)
      t2[k] = make_float2(static_cast<float>(r[j].o[2 * k]), static_cast<float>(r[j].o[2 * k + 1]));
  }
  wave_lds_sync();
  wave_copy_rows(wtile, dst, nrows);
  wave_lds_sync();
}

// A wave's nrows x 10 fp32 LDS slice to dst: 16-byte stores when dst allows, else 8-byte.
__device__ __forceinline__ void wave_copy_rows(const float* wtile, float* dst, int nrows) {
  const int lane = threadIdx.x & 63;
  // a full wave (64 rows = 160 16-byte pieces) into a 16-byte aligned destination: three fixed
  // lane passes instead of the strided loop (wave-uniform test)
  if (dst != nullptr && nrows == 64 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    f32x4* d4 = reinterpret_cast<f32x4*>(dst);
    const f32x4* s4 = reinterpret_cast<const f32x4*>(wtile);
    const f32x4 v0 = s4[lane], v1 = s4[64 + lane];
    const f32x4 v2 = s4[128 + (lane & 31)];
    st_out(d4 + lane, v0);
    st_out(d4 + 64 + lane, v1);
    if (lane < 32) st_out(d4 + 128 + lane, v2);
    return;
  }
  if (dst != nullptr && nrows > 0) {
    const int nfl = nrows * kObs;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      const int n4 = nfl >> 2;
      f32x4* d4 = reinterpret_cast<f32x4*>(dst);
      const f32x4* s4 = reinterpret_cast<const f32x4*>(wtile);
      for (int j = lane; j < n4; j += 64) st_out(d4 + j, s4[j]);
      const int tail = nfl - (n4 << 2);
      if (lane < tail) st_out(dst + (n4 << 2) + lane, wtile[(n4 << 2) + lane]);
    } else {
      const int n2 = nfl >> 1;
      f32x2* d2 = reinterpret_cast<f32x2*>(dst);
      const f32x2* s2 = reinterpret_cast<const f32x2*>(wtile);
      for (int j = lane; j < n2; j += 64) st_out(d2 + j, s2[j]);
    }
  }
}

// Step t's won bits of one wave (every lane calls it): word t * ceil(n/64) + wbase / 64.
__device__ __forceinline__ void store_won_mask(uint64_t* mask, bool won, int t, int64_t n,
                                               int64_t wbase, int wrows) {
  if (mask == nullptr) return;
  const uint64_t m = __ballot(won);
  if ((threadIdx.x & 63) == 0 && wrows > 0)
    st_out(mask + static_cast<int64_t>(t) * ((n + 63) >> 6) + (wbase >> 6), m);
}

// The env index through an empty asm: the state stores recompute their addresses from it
// instead of keeping the load addresses (two VGPRs per array) live across the step.
__device__ __forceinline__ int64_t opaque_index(int64_t i) {
  asm volatile("" : "+v"(i));
  return i;
}

// One env-step's four byte outputs (a1, a2, done, collision) as the little-endian u32 of an
// interleaved [.., 4] uint8 buffer (mg_outputs.flags, mg_traj.flags).
MG_HD uint32_t pack_step_bytes(int a1, int a2, bool done, bool coll) {
  return static_cast<uint32_t>(a1 & 0xff) | (static_cast<uint32_t>(a2 & 0xff) << 8) |
         (done ? 0x10000u : 0u) | (coll ? 0x1000000u : 0u);
}

struct Launch {
  mg_params P;
  Reset0 R0;
  mg_state S;
  mg_outputs O;
  mg_stats St;
  const int8_t* a1;
  const int8_t* a2;
  int8_t* a1_out;
  int8_t* a2_out;
  uint64_t seed;
  uint64_t step_idx;
  int64_t env_offset;
  int64_t n;
  uint32_t flags;
  int32_t opp_random;
};

// The step kernel. OUT64 = the single-env path (packed fp64 record, no LDS staging).
template <int ACT, bool OUT64>
__global__ __launch_bounds__(kBlock) void step_kernel(const Launch L) {
  __shared__ __attribute__((aligned(16))) float obs_tile[kBlock * kObs];

  const mg_params& P = L.P;
  const int tid = threadIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock;
  const int64_t i = base + tid;
  const bool live = i < L.n;
  StepOut r;
  r.done = false;
  bool won = false;

  if (live) {
    int a1, a2;
    if constexpr (ACT == kActPhilox) {
      draw_actions(static_cast<uint64_t>(L.env_offset + i), L.step_idx, L.seed, L.opp_random, a1, a2);
      if (!L.O.flags) {  // with O.flags the actions go out with done / collision below
        if (L.a1_out) st_out(L.a1_out + i, static_cast<int8_t>(a1));
        if (L.a2_out) st_out(L.a2_out + i, static_cast<int8_t>(a2));
      }
    } else {
      a1 = L.a1[i];
      a2 = L.a2 ? static_cast<int>(L.a2[i]) : MG_ACTION_NONE;
    }
    // the two action_dict lookups (vector loads from the launch arguments) issued before the
    // state loads, so they are in flight together (looked up inside the step, the first one's
    // wait came after the state had arrived): -1 to -1.5 % per launch (r03q)
    const double sp1 = action_speed_or0(P, a1), sp2 = action_speed_or0(P, a2);
    Env e = load_env(L.S, i);
    env_step_sp(P, e, a1, a2, sp1, sp2, r);
    if (r.bad) {
      if (L.O.error) atomicOr(L.O.error, r.bad);
      store_env(L.S, i, e);  // clock (and the ego for a bad action2) advanced, nothing else
    } else {
      if constexpr (OUT64) {
        mg_rec64* rec = L.O.rec64 + i;
        {  // the fp64 observation of the state after the step (score_step's values, recomputed)
          double x1, y1, x2, y2, od[kObs];
          lon2coord(P, e.p1, true, x1, y1);
          lon2coord(P, e.p2, false, x2, y2);
          observe(P, e.p1, e.v1, e.p2, e.v2, x1, y1, x2, y2, od);
#pragma unroll
          for (int k = 0; k < kObs; ++k) rec->obs[k] = od[k];
        }
        rec->rew[0] = r.r1;
        rec->rew[1] = r.r2;
        rec->acc[0] = r.acc1;
        rec->acc[1] = r.acc2;
        rec->pos[0] = e.p1;
        rec->pos[1] = e.p2;
        rec->vel[0] = e.v1;
        rec->vel[1] = e.v2;
        rec->ret[0] = e.ret1;
        rec->ret[1] = e.ret2;
        rec->tf = pack_tf(e);
        rec->status = (r.done ? MG_ST_DONE : 0u) | (r.coll ? MG_ST_COLLISION : 0u) |
                      (r.r1_int ? MG_ST_R1_INT : 0u) | (r.r2_int ? MG_ST_R2_INT : 0u) |
                      (r.v1_int ? MG_ST_V1_INT : 0u) | (r.v2_int ? MG_ST_V2_INT : 0u);
      } else if (L.O.rew) {
        st_out(reinterpret_cast<f32x2*>(L.O.rew) + i,
               f32x2{static_cast<float>(r.r1), static_cast<float>(r.r2)});
      }
      if (L.O.flags) {
        st_out(reinterpret_cast<uint32_t*>(L.O.flags) + i, pack_step_bytes(a1, a2, r.done, r.coll));
      } else {
        if (L.O.done) st_out(L.O.done + i, static_cast<uint8_t>(r.done ? 1 : 0));
        if (L.O.coll) st_out(L.O.coll + i, static_cast<uint8_t>(r.coll ? 1 : 0));
      }
      won = e.winner == 1;
      // statistics by read-modify-write: the no-wait atomics (finish_episode_nowait) measured
      // +4 % per launch here at 2^20 (r04j), where the finishing lanes' loads hit the Infinity Cache
      after_step(P, e, r, L.St, L.O.final_obs ? L.O.final_obs + i * kObs : nullptr, i,
                 (L.flags & MG_AUTORESET) != 0, nullptr, &L.R0);
      store_env(L.S, opaque_index(i), e);
    }
  }

  if (L.O.done_mask) {
    const uint64_t m = __ballot(live && r.done);
    if ((tid & 63) == 0 && live) L.O.done_mask[i >> 6] = m;
  }
  if (L.O.won_mask) {
    const uint64_t m = __ballot(won);
    if ((tid & 63) == 0 && live) L.O.won_mask[i >> 6] = m;
  }
  if constexpr (!OUT64) {
    // per-wave staging, no block barrier: a wave held up by a finishing lane's statistics
    // read-modify-write (a DRAM read past the Infinity Cache) no longer holds up the block's
    // other three at the barrier (2^22 envs: 107.0 -> 104.8 us per launch with the lookups
    // above, r03q; +-0 at 2^20)
    if (L.O.obs) {
      const int64_t wbase = base + (tid & ~63);
      const int64_t wrem = L.n - wbase;
      wave_store_obs(obs_tile + (tid & ~63) * kObs, r.o, L.O.obs + wbase * kObs,
                     wrem <= 0 ? 0 : (wrem < 64 ? static_cast<int>(wrem) : 64));
    }
  }
}

// One env-step's four byte outputs of a trajectory (a1, a2, done, collision): a single 32-bit
// store into the interleaved [T, n, 4] buffer when the caller gave one, else four byte stores.
__device__ __forceinline__ void store_step_bytes(const mg_traj& T, int64_t row, int a1, int a2, bool done,
                                                 bool coll) {
  if (T.flags) {
    st_out(reinterpret_cast<uint32_t*>(T.flags) + row, pack_step_bytes(a1, a2, done, coll));
    return;
  }
  if (T.a1) st_out(T.a1 + row, static_cast<int8_t>(a1));
  if (T.a2) st_out(T.a2 + row, static_cast<int8_t>(a2));
  if (T.done) st_out(T.done + row, static_cast<uint8_t>(done ? 1 : 0));
  if (T.coll) st_out(T.coll + row, static_cast<uint8_t>(coll ? 1 : 0));
}

struct Rollout {
  mg_params P;
  Reset0 R0;
  mg_state S;
  mg_traj T;
  mg_stats St;
  uint64_t seed;
  uint64_t first_step;
  int64_t env_offset;
  int64_t n;
  int32_t num_steps;
  int32_t opp_random;
  uint32_t flags;
};

// num_steps consecutive mg_step_random steps with the env kept in registers: the state is
// read once and written once per launch; step t's outputs go to slice t of the trajectory.
// FULL: the outputs every MergeVecEnv rollout passes are present (obs, rew, the interleaved step
// record, statistics, autoreset; final observations and the won mask stay optional). The
// instance assumes so, which drops null tests the compiler otherwise keeps live across the loop
// as 64-bit lane masks (SGPR pairs, spilled into VGPR lanes: a v_readlane per use).
template <bool FULL>
__global__ __launch_bounds__(kBlock) void rollout_kernel(const Rollout R) {
  __shared__ __attribute__((aligned(16))) float obs_tile[kBlock * kObs];

  if constexpr (FULL) {
    __builtin_assume(R.T.obs != nullptr);
    __builtin_assume(R.T.rew != nullptr);
    __builtin_assume(R.T.flags != nullptr);
    __builtin_assume(R.St.rec != nullptr);
    __builtin_assume((R.flags & MG_AUTORESET) != 0);
  }
  const mg_params& P = R.P;
  const int tid = threadIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock;
  const int64_t i = base + tid;
  const bool live = i < R.n;
  const int64_t wbase = base + (tid & ~63);
  const int64_t wrem = R.n - wbase;
  const int wrows = wrem <= 0 ? 0 : (wrem < 64 ? static_cast<int>(wrem) : 64);
  const bool autoreset = (R.flags & MG_AUTORESET) != 0;

  Env e;
  // statistics in registers for the launch: -9.5 % per step against the read-modify-write (the
  // finishing lanes no longer wait on a load); the no-wait atomics measured +16 % median (r04j)
  EpStats sreg;
  if (live) {
    e = load_env(R.S, i);
    stats_load(R.St, i, sreg);
  }
  bool won = false;
  uint4 u = make_uint4(0u, 0u, 0u, 0u);  // the Philox block of the current eight steps
  for (int t = 0; t < R.num_steps; ++t) {
    StepOut r;  // per step: no loop-carried copy of the observation (dead lanes store nothing)
    const int64_t row = static_cast<int64_t>(t) * R.n + i;
    const uint64_t k = R.first_step + t;
    if (t == 0 || k % kStepsPerPhilox == 0)  // wave-uniform
      u = philox_block(static_cast<uint64_t>(R.env_offset + i), k / kStepsPerPhilox, R.seed, /*opaque_key=*/true);
    if (live) {
      int a1, a2;
      actions_from_block(u, k, R.opp_random, a1, a2);
      env_step<false>(P, e, a1, a2, r);  // Philox actions are always valid: the unchecked step
      if (R.T.rew)
        st_out(reinterpret_cast<f32x2*>(R.T.rew) + row,
               f32x2{static_cast<float>(r.r1), static_cast<float>(r.r2)});
      store_step_bytes(R.T, row, a1, a2, r.done, r.coll);
      won = e.winner == 1;
      after_step(P, e, r, R.St, R.T.final_obs ? R.T.final_obs + row * kObs : nullptr, i, autoreset, &sreg, &R.R0);
    }
    store_won_mask(R.T.won_mask, won, t, R.n, wbase, wrows);
    if (R.T.obs)  // staged per wave: waves never wait for each other
      wave_store_obs(obs_tile + (tid & ~63) * kObs, r.o,
                     R.T.obs + (static_cast<int64_t>(t) * R.n + wbase) * kObs, wrows);
  }
  if (live) {
    store_env(R.S, i, e);
    stats_store(R.St, i, sreg);
  }
}

// ============================================================================ Q-net policy
// The reference's DQN Net (scripts/main.py:30-47, scripts/hdqn.py:38-55): Linear(in,200) ->
// ReLU -> Linear(200,100) -> ReLU -> Linear(100,out), and its epsilon-greedy choose_action
// (main.py:99-112: greedy argmax when np.random.randn() <= EPISILO, else uniform). Computed
// in bf16 on the matrix cores with fp32 accumulation, one wave per 64 envs, in the TRANSPOSED
// form  H1' = W1 X',  H2' = W2 H1',  Q' = W3 H2'  (hidden units on tile rows, envs on lanes):
//  * layer 1 (K = 16: up to 13 inputs and the 3 bias slots) on v_mfma_f32_32x32x16_bf16, 7 row
//    tiles of 32 units x 2 column tiles of 32 envs;
//  * layers 2 and 3 on v_mfma_f32_16x16x32_bf16: H2' in 7 row tiles of 16 units x 4 column tiles
//    of 16 envs over 7 k-blocks of 32 hidden-1 units, Q' in one row tile over 4 k-blocks of 32
//    hidden-2 units. Under load the chip holds a higher clock for the 16x16 shape at equal cycles
//    per FLOP (tools/micro/qfwd_probe.hip: 2.33-2.47 PF against 2.07 PF for 32x32x16, r03ab), and
//    16-row tiles pad hidden-2 to 112 units instead of 128: 14 x 32 + (196 + 16) x 16 = 3,840
//    matrix cycles per 64-env forward (round 3's all-32x32 forward: 132 x 32 = 4,224).
// No layer's output goes through LDS:
//  * a 32x32 layer-1 accumulator holds its 32 envs (lane & 31) in both lane halves. After ReLU +
//    bf16 packing, one v_permlane16_swap per pair of packed registers leaves envs 0..15 in every
//    16-lane row of the first register and envs 16..31 in the second: each is then the B operand
//    of a 16x16x32 MFMA (lane l: env column l & 15, k = 8 (l >> 4) + j), in the k order
//    qnet_unit1, which mg_qnet_pack gives W2's columns;
//  * a 16x16 accumulator holds rows 4 (l >> 4) .. + 3 of column l & 15, so two row tiles side by
//    side are the B operand of a layer-3 k-block (k order qnet_unit2, W3's columns);
//  * the Q tiles of the four column tiles reach one env per lane through two v_permlane32_swap and
//    one v_permlane16_swap per register (qnet_gather_q).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kQH1Real = 200, kQH2Real = 100;  // main.py:30-47 Net widths
constexpr int kQT1 = 7;  // layer-1 row tiles of 32 units = layer-2 k-blocks (224 >= 203)
constexpr int kQT2 = 7;  // layer-2 row tiles of 16 units (112 >= 103)
constexpr int kQK3 = 4;  // layer-3 k-blocks of 32 hidden-2 units (two row tiles each)
// Biases are folded into the padded K slots: each bias b is split into three bf16 parts
// hi + mid + lo == b exactly (8 significant bits each, 24 = fp32's), stored as three weight
// columns whose inputs are 1.0 -- layer-1 inputs 13..15, hidden-1 units 200..202 and hidden-2
// units 100..102 (W1 / W2 rows that output exactly 1.0). The matrix cores add the fp32 bias
// inside the K sum, so there are no bias loads and every accumulator starts at an inline zero
// (a bias-initialised accumulator cost 4 ds_read_b128 per tile and the zeroing or bias moves;
// folding measured -5..8 % on the config-5 kernel). Summation order is the only difference.
constexpr int kQBiasIn = 13;       // first of the three layer-1 input slots holding 1.0
constexpr int kQOne1 = 200;        // hidden-1 units 200..202 = 1.0
constexpr int kQOne2 = 100;        // hidden-2 units 100..102 = 1.0
constexpr int kQMaxIn = kQBiasIn;  // widest net input: 13
static_assert(32 * kQT1 >= kQOne1 + 3 && 32 * (kQT1 - 1) < kQH1Real && 16 * kQT2 >= kQOne2 + 3 &&
                  16 * (kQT2 - 1) < kQH2Real && 32 * kQK3 >= 16 * kQT2,
              "tile counts cover the hidden units and their 1.0 units, no tile is all padding");
// specialised kernel: 4 Q-net waves + kQWsEnvWaves env waves (8 env waves -- 3 waves per SIMD,
// a Q-net wave within 168 VGPRs -- measured 19 % slower); each env lane steps kQWsIlp envs per
// phase, in lockstep (independent fp64 chains interleaved in one instruction stream), so a group
// is 64 x env waves x ILP envs and a block holds two
constexpr int kQWsEnvWaves = 4;
constexpr int kQWsIlp = 2;
constexpr int kQWsThreads = 64 * (4 + kQWsEnvWaves);
constexpr int kQWsWavesPerSimd = (4 + kQWsEnvWaves) / 4;

// The packed net (mg_qnet_pack) is the forward's MFMA A operands in the order it consumes them,
// each fragment the 64 lanes' 16 bytes contiguous, so a wave's ds_read_b128 (LDS nets) or
// buffer_load_dwordx4 (nets read from L2) covers 1 KB of consecutive bytes: conflict-free in LDS,
// 8 cache lines from L2. Consumption order:
//   s = 0: W1(0); for k-block kb = 0..5: W1(kb + 1), then W2(t, kb) for row tiles t = 0..6;
//   kb = 6 interleaved with layer 3:  W2(0,6) W2(1,6) W2(2,6) W3(0) W2(3,6) W2(4,6) W3(1)
//                                     W2(5,6) W2(6,6) W3(2) W3(3)
// W1(m): lane l = 32 h + r holds W1[32 m + r][8 h .. 8 h + 7] (inputs in natural order, b1's parts
// at 13..15). W2(t, kb): lane l holds row 16 t + (l & 15), hidden-1 units qnet_unit1(kb, l >> 4,
// j = 0..7). W3(kb): 512 B -- output rows 0..7 only; lane l reads row l & 7, so rows 8..15 of the
// Q tile repeat rows 0..7 and are never read.
struct QFrag {
  int kind, tile, kb;  // kind 0: W1(tile), 1: W2(tile, kb), 2: W3(kb)
};
constexpr int kQFrags = 1 + 6 * 8 + 11;
// Closed forms (no loops or tables), so that every fragment offset of the unrolled forward folds
// to a constant. Last k-block: entry u = s - 49 is W3 at u = 3, 6, 9, 10, else W2 row tile u - u / 3.
__host__ __device__ constexpr QFrag qfrag(int s) {
  if (s == 0) return QFrag{0, 0, 0};
  if (s < 49) {
    const int u = s - 1, kb = u / 8, v = u % 8;
    return v == 0 ? QFrag{0, kb + 1, 0} : QFrag{1, v - 1, kb};
  }
  const int u = s - 49;
  if (u == 10) return QFrag{2, 0, 3};
  return u % 3 == 0 && u > 0 ? QFrag{2, 0, u / 3 - 1} : QFrag{1, u - u / 3, kQT1 - 1};
}
__host__ __device__ constexpr int qfrag_off(int s) {
  if (s <= 49) return 1024 * s;
  const int u = s - 49;
  return 1024 * s - 512 * ((u > 3) + (u > 6) + (u > 9) + (u > 10));
}
constexpr int kQNetBytes = qfrag_off(kQFrags);  // 59,392 B
static_assert(kQNetBytes == 56 * 1024 + 4 * 512, "7 W1 + 49 W2 fragments of 1 KB, 4 W3 of 512 B");

// hidden-1 unit at k = 8 g + j of layer-2 k-block kb: 32x32 accumulator register i = 2 q + e of
// lane half h holds row (i & 3) + 8 (i >> 2) + 4 h; after the swap, lane row g holds packed
// register q + 4 (g & 1) of half g >> 1 as its dword q
__host__ __device__ constexpr int qnet_unit1(int kb, int g, int j) {
  return 32 * kb + (j & 3) + 8 * (j >> 2) + 16 * (g & 1) + 4 * (g >> 1);
}
// hidden-2 unit at k = 8 g + j of layer-3 k-block kb: rows 4 g .. 4 g + 3 of row tiles 2 kb
// (j < 4) and 2 kb + 1 (j >= 4)
__host__ __device__ constexpr int qnet_unit2(int kb, int g, int j) {
  return 32 * kb + 16 * (j >> 2) + 4 * g + (j & 3);
}

// ReLU + bf16 pack of two accumulator values: one v_cvt_pk_bf16_f32 + one v_pk_max_i16
// (a 2-wide fptrunc selects ONE convert; scalar casts cost 2 converts + a perm). Rounded first,
// then max(x, 0) on the packed bf16 pairs as signed 16-bit integers: a bf16 with its sign bit set
// is a negative int16 (and -0.0 becomes +0.0), so max_i16(x, 0) is exactly ReLU.
__device__ __forceinline__ uint32_t relu_pair(float x, float y) {
  i16x2 v = __builtin_bit_cast(i16x2, __builtin_convertvector(f32x2{x, y}, bf16x2));
  const i16x2 zero = {0, 0};
  v = __builtin_elementwise_max(v, zero);
  return __builtin_bit_cast(uint32_t, v);
}

// Layer-1 B fragment of one env: features k = 8h .. 8h+7 of its observation row, in the
// swapped order state[5:] + state[:5] when swap (main.py:199); features 8..15 are x8, x9, 0, 0,
// 0, 1, 1, 1 (the 1.0 inputs of b1's three parts). The row is read with five unconditional
// ds_read_b64 and converted pairwise; the lane half picks its pairs with selects (per-element
// conditional loads cost a full LDS wait each).
__device__ __forceinline__ bf16x8 qnet_input(const float* row, bool swap, int h) {
  float v[kObs];
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k) {
    const f32x2 t = reinterpret_cast<const f32x2*>(row)[k];
    v[2 * k] = t[0];
    v[2 * k + 1] = t[1];
  }
  uint32_t pr[kObs / 2];
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k) {
    const int a = swap ? (2 * k + 5) % kObs : 2 * k, b = swap ? (2 * k + 6) % kObs : 2 * k + 1;
    pr[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[a], v[b]}, bf16x2));
  }
  static_assert(kQBiasIn == 13 && kObs == 10, "bias slots 13..15 follow the 10 features");
  const u32x4 w = h ? u32x4{pr[4], 0u, 0x3F800000u, 0x3F803F80u} : u32x4{pr[0], pr[1], pr[2], pr[3]};
  return __builtin_bit_cast(bf16x8, w);
}

// Layer-1 B fragment from a 16-float row (in_dim <= 13, zero padded, 1.0 at 13..15): features
// 8h .. 8h+7. The standalone forward takes any input width this way, e.g. hdqn.py's goal states
// [goal] + state (11 values, :291) for its lower-level Net(NUM_STATES + 1, NUM_ACTIONS) (:145).
__device__ __forceinline__ bf16x8 qnet_input_wide(const float* row16, int h) {
  const f32x4 lo = reinterpret_cast<const f32x4*>(row16 + 8 * h)[0];
  const f32x4 hi = reinterpret_cast<const f32x4*>(row16 + 8 * h)[1];
  const u32x4 w = {__builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo[0], lo[1]}, bf16x2)),
                   __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo[2], lo[3]}, bf16x2)),
                   __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{hi[0], hi[1]}, bf16x2)),
                   __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{hi[2], hi[3]}, bf16x2))};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Packs fp32 torch Linear weights (row-major [out][in]) and biases into the fragment layout above:
// one thread per (fragment, lane, element).
__global__ void qnet_pack_kernel(const float* w1, const float* b1, const float* w2, const float* b2,
                                 const float* w3, const float* b3, int in_dim, int out_dim,
                                 uint8_t* packed) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kQFrags * 64 * 8) return;
  const int s = e >> 9, lane = (e >> 3) & 63, j = e & 7;
  const QFrag f = qfrag(s);
  // part p (0 hi, 1 mid, 2 lo) of the three-way bf16 split of b (hi + mid + lo == b)
  auto part = [](float b, int p) {
    const float hi = static_cast<float>(static_cast<__bf16>(b));
    const float r = b - hi;
    const float mid = static_cast<float>(static_cast<__bf16>(r));
    return p == 0 ? hi : p == 1 ? mid : r - mid;
  };
  float v = 0.f;
  int off = qfrag_off(s) + 16 * lane;
  if (f.kind == 0) {  // W1[m][k]: the input features, then b1's parts; hidden-1 units 200..202 = 1.0
    const int m = 32 * f.tile + (lane & 31), k = 8 * (lane >> 5) + j;
    if (m < kQH1Real && k < in_dim) v = w1[m * in_dim + k];
    else if (m < kQH1Real && k >= kQBiasIn && k < kQBiasIn + 3) v = part(b1[m], k - kQBiasIn);
    else if (m >= kQOne1 && m < kQOne1 + 3 && k == kQBiasIn) v = 1.f;
  } else if (f.kind == 1) {  // W2[m][u], u = qnet_unit1: then b2's parts; hidden-2 units 100..102 = 1.0
    const int m = 16 * f.tile + (lane & 15), u = qnet_unit1(f.kb, lane >> 4, j);
    if (m < kQH2Real && u < kQH1Real) v = w2[m * kQH1Real + u];
    else if (m < kQH2Real && u >= kQOne1 && u < kQOne1 + 3) v = part(b2[m], u - kQOne1);
    else if (m >= kQOne2 && m < kQOne2 + 3 && u == kQOne1) v = 1.f;
  } else {  // W3[m][u], u = qnet_unit2, then b3's parts; rows 0..7 of 16
    if ((lane & 15) >= 8) return;
    const int m = lane & 7, u = qnet_unit2(f.kb, lane >> 4, j);
    if (m < out_dim && u < kQH2Real) v = w3[m * kQH2Real + u];
    else if (m < out_dim && u >= kQOne2 && u < kQOne2 + 3) v = part(b3[m], u - kQOne2);
    off = qfrag_off(s) + 16 * (8 * (lane >> 4) + m);
  }
  reinterpret_cast<__bf16*>(packed + off)[j] = static_cast<__bf16>(v);
}

// A zero the compiler cannot see through. Added to the LDS addresses of loop-invariant
// weight loads so they are issued where they are used: hoisted out of the tile and time loops,
// they stay live across them and push the kernel into scratch.
__device__ __forceinline__ int opaque_zero() {
  int z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// Cooperative copy of a packed net into LDS (all threads of the block; caller syncs).
__device__ __forceinline__ void qnet_to_lds(const uint8_t* net, uint8_t* lds) {
  const f32x4* src = reinterpret_cast<const f32x4*>(net);
  f32x4* dst = reinterpret_cast<f32x4*>(lds);
  for (int j = threadIdx.x; j < kQNetBytes / 16; j += blockDim.x) dst[j] = src[j];
}

// Fragment s of a packed net for this lane: a net in LDS ...
struct QSrcLds {
  const uint8_t* net;  // + opaque zero: the loads stay where they are used
  int lo, lo3;         // lane byte offsets within a W1 / W2 fragment and within a W3 fragment
  __device__ __forceinline__ bf16x8 operator()(int s) const {
    return *reinterpret_cast<const bf16x8*>(net + qfrag_off(s) + (qfrag(s).kind == 2 ? lo3 : lo));
  }
};
// ... or in global memory (the h-DQN kernel's opponent from another checkpoint: four nets exceed
// one CU's LDS, so the opponent's two are read from L2), through a buffer resource: the lane offset
// in a VGPR, the fragment's offset a constant
struct QSrcGlobal {
  __amdgpu_buffer_rsrc_t rs;
  int lo, lo3;
  __device__ __forceinline__ bf16x8 operator()(int s) const {
    return __builtin_bit_cast(
        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, qfrag(s).kind == 2 ? lo3 : lo, qfrag_off(s), 0));
  }
};
__device__ __forceinline__ int qnet_lane_off() { return 16 * (threadIdx.x & 63); }
__device__ __forceinline__ int qnet_lane_off3() {
  const int lane = threadIdx.x & 63;
  return 16 * (8 * (lane >> 4) + (lane & 7));
}
__device__ __forceinline__ QSrcLds qnet_lds(const uint8_t* net) {
  return QSrcLds{net + opaque_zero(), qnet_lane_off(), qnet_lane_off3()};
}
__device__ __forceinline__ QSrcGlobal qnet_global(const uint8_t* net) {
  // gfx9 buffer descriptor word 3 (raw untyped dword access), num_records = the packed net
  return QSrcGlobal{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(net), static_cast<short>(0), kQNetBytes,
                                                      0x00020000),
                    qnet_lane_off(), qnet_lane_off3()};
}
constexpr int kQLdsAhead = 2;     // fragments in flight, LDS nets
constexpr int kQGlobalAhead = 3;  // fragments in flight, nets read from L2 (five measured the same, r03e)

// (x, y) -> (x with y's lane rows swapped in as documented for the instruction, y likewise).
// Operands into locals and the result read as one 64-bit value: hipcc (ROCm 7.2) passed element 0
// for every j when the builtin's arguments were subscripts, and returned the first result for
// both subscripts of its 2-vector.
__device__ __forceinline__ void permlane16_swap(uint32_t& x, uint32_t& y) {
  const uint32_t a = x, b = y;
  const uint64_t sw = __builtin_bit_cast(uint64_t, __builtin_amdgcn_permlane16_swap(a, b, false, false));
  x = static_cast<uint32_t>(sw);
  y = static_cast<uint32_t>(sw >> 32);
}

// Q tile of column tile t: lane row g holds rows 4 g + i of env 16 t + (l & 15) in register i.
// Transposed over (g, t) so that lane l = 16 g + c ends with rows 0..7 of env 16 g + c = l:
// permlane32_swap of tiles (0, 2) and (1, 3) leaves rows 0-3 / 4-7 of tiles 0 and 2 (resp. 1, 3)
// in lane rows 0, 1, 2, 3 of the first register; permlane16_swap of those two registers then gives
// rows 0-3 of tile g in lane row g of the first and rows 4-7 in the second.
__device__ __forceinline__ void qnet_gather_q(const f32x4 (&acc3)[4], float (&q)[8]) {
  // Inline asm: with the builtins, hipcc (ROCm 7.2) computed register 0's swaps only and returned
  // them for all four registers. The compiler does not pad hazards inside inline asm, and the
  // operands come straight from the last layer-3 MFMAs (VGPR accumulators in the rollout kernels):
  // 16 wait states first cover the XDL-write -> VALU-read distance of a 16x16x32 result (and the
  // two a VALU write needs before a swap reads it), two more after the block.
  float x0[4], y0[4], x1[4], y1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x0[i] = acc3[0][i];
    y0[i] = acc3[2][i];
    x1[i] = acc3[1][i];
    y1[i] = acc3[3][i];
  }
  asm volatile(
      "s_nop 7\n\ts_nop 7\n\t"
      "v_permlane32_swap_b32 %0, %4\n\tv_permlane32_swap_b32 %8, %12\n\t"
      "v_permlane32_swap_b32 %1, %5\n\tv_permlane32_swap_b32 %9, %13\n\t"
      "v_permlane32_swap_b32 %2, %6\n\tv_permlane32_swap_b32 %10, %14\n\t"
      "v_permlane32_swap_b32 %3, %7\n\tv_permlane32_swap_b32 %11, %15\n\t"
      "s_nop 1\n\t"
      "v_permlane16_swap_b32 %0, %8\n\tv_permlane16_swap_b32 %1, %9\n\t"
      "v_permlane16_swap_b32 %2, %10\n\tv_permlane16_swap_b32 %3, %11\n\t"
      "s_nop 1"
      : "+v"(x0[0]), "+v"(x0[1]), "+v"(x0[2]), "+v"(x0[3]), "+v"(y0[0]), "+v"(y0[1]), "+v"(y0[2]), "+v"(y0[3]),
        "+v"(x1[0]), "+v"(x1[1]), "+v"(x1[2]), "+v"(x1[3]), "+v"(y1[0]), "+v"(y1[1]), "+v"(y1[2]), "+v"(y1[3]));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    q[i] = x0[i];
    q[4 + i] = x1[i];
  }
}

// Q-values of this lane's env row0 + lane (rows 0..7) from the layer-1 B fragments of the wave's
// two 32-env column tiles (xb0: envs row0 + r, xb1: envs row0 + 32 + r, k-half h = lane >> 5),
// with the weight fragments from src, D in flight. Every lane of the wave must call it.
// Software-pipelined and fully unrolled: layer 1 of k-block kb + 1 is issued ahead of layer 2 of
// k-block kb, and its ReLU, packing and swaps are computed in pieces between kb's layer-2 MFMAs
// (each W2 fragment feeds the four column tiles' MFMAs); layer 3's k-blocks follow the last
// k-block's layer-2 row tiles they read. Unrolled, the first MFMA into each accumulator takes an
// inline zero and the next k-block's operands land in their final registers.
//
// NC (round 5): the number of 16-env column tiles computed, 1..4: lanes 16 NC .. 63 get no result.
// Column tiles are independent (each MFMA column is one env), so the envs computed get the same
// bits as in a full forward; a pass over a compacted list of the envs whose Q the reference
// evaluates (its greedy branch) skips the other tiles' MFMAs. NC <= 2 also skips the layer-1 half
// xb1 and its ReLU / swap work. A compile-time count (qnet_mlp_nc dispatches): guarding each MFMA
// with a runtime test put a scalar branch behind every MFMA and cost +66 % per h-DQN launch even
// where every tile ran (r05a).
template <int D, int NC = 4, class Src>
__device__ __forceinline__ void qnet_mlp(const Src& src, bf16x8 xb0, bf16x8 xb1, float (&q)[8]) {
  static_assert(NC >= 1 && NC <= 4, "1..4 column tiles");
  constexpr int nc = NC;
  static_assert(kQT1 == 7 && kQT2 == 7 && kQK3 == 4 && kQFrags == 60,
                "qfrag's consumption order assumes 7 k-blocks, 7 layer-2 row tiles and 4 layer-3 k-blocks");
  bf16x8 ring[D];
#pragma unroll
  for (int s = 0; s < D; ++s) ring[s] = src(s);
  auto take = [&](int s) __attribute__((always_inline)) {
    const bf16x8 f = ring[s % D];
    if (s + D < kQFrags) ring[s % D] = src(s + D);
    return f;
  };
  const f32x16 z16 = {};
  const f32x4 z4 = {};
  f32x16 c0, c1;
  constexpr bool hi = nc > 2;  // column tiles 2 and 3: the layer-1 half xb1
  auto layer1 = [&](int s) __attribute__((always_inline)) {
    const bf16x8 a1 = take(s);
    c0 = mfma32(a1, xb0, z16);
    if (hi) c1 = mfma32(a1, xb1, z16);
  };
  // packed ReLU pairs of c0 (d = 0..7) and c1 (d = 8..15)
  auto relu_d = [&](int d) __attribute__((always_inline)) {
    const f32x16& c = d < 8 ? c0 : c1;
    const int b = 2 * (d & 7);
    return relu_pair(c[b], c[b + 1]);
  };
  uint32_t nx[16];
  // swaps of column tile u's packed registers: afterwards nx[8u + q] is dword q of the B operand
  // of env tile 2u, nx[8u + 4 + q] that of env tile 2u + 1
  auto swap_u = [&](int u) __attribute__((always_inline)) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) permlane16_swap(nx[8 * u + qd], nx[8 * u + 4 + qd]);
  };
  auto operands = [&](bf16x8 (&hb)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t) hb[t] = __builtin_bit_cast(bf16x8, u32x4{nx[4 * t], nx[4 * t + 1], nx[4 * t + 2], nx[4 * t + 3]});
  };
  layer1(0);
#pragma unroll
  for (int d = 0; d < 8; ++d) nx[d] = relu_d(d);
  if (hi) {
#pragma unroll
    for (int d = 8; d < 16; ++d) nx[d] = relu_d(d);
  }
  swap_u(0);
  if (hi) swap_u(1);
  bf16x8 hb[4];
  operands(hb);
  f32x4 acc2[kQT2][4];
  // One MFMA per slot and the vector work placed behind it, in source order (sched_barrier): a
  // 16x16x32 MFMA occupies the matrix pipe 16 cycles, room for one ReLU pair (v_cvt_pk + v_pk_max)
  // or one swap of the wave's own instruction stream; left to the scheduler, the four MFMAs of a
  // row tile went out back to back and the vector work behind them held the next row tile.
  auto slot = [&](f32x4& acc, const bf16x8& a, const bf16x8& b, bool zero) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma16(a, b, zero ? z4 : acc);
  };
  int s = 1;
#pragma unroll
  for (int kb = 0; kb < kQT1 - 1; ++kb) {
    layer1(s++);
#pragma unroll
    for (int t2 = 0; t2 < kQT2; ++t2) {
      const bf16x8 a2 = take(s++);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nc) slot(acc2[t2][t], a2, hb[t], kb == 0);
        // the next k-block's operands: ReLU pairs behind row tiles 1..4, swaps behind 5 and 6
        if (t2 >= 1 && t2 <= 4 && (t2 <= 2 || hi)) nx[4 * (t2 - 1) + t] = relu_d(4 * (t2 - 1) + t);
        if (t2 == 5) permlane16_swap(nx[t], nx[4 + t]);
        if (t2 == 6 && hi) permlane16_swap(nx[8 + t], nx[12 + t]);
      }
    }
    operands(hb);
  }
  // The last k-block with layer 3 interleaved. Layer-3 k-block k3 reads row tiles 2 k3 and 2 k3 + 1;
  // the ReLU pairs of its B operands are built in the slots after each row tile's MFMAs have issued
  // (two pairs per slot), into two buffers used alternately.
  f32x4 acc3[4] = {z4, z4, z4, z4};  // the tiles past nc stay zero (never read as results)
  uint32_t b3[2][4][4];
  auto pairs3 = [&](int t2, int t) __attribute__((always_inline)) {  // row tile t2 of env tile t
    const int buf = (t2 >> 1) & 1, d = 2 * (t2 & 1);
    b3[buf][t][d] = relu_pair(acc2[t2][t][0], acc2[t2][t][1]);
    b3[buf][t][d + 1] = relu_pair(acc2[t2][t][2], acc2[t2][t][3]);
  };
  // slots of layer-2 row tile t2, each followed by the pairs of row tile p (p < 0: none)
  auto layer2 = [&](int t2, int p) __attribute__((always_inline)) {
    const bf16x8 a2 = take(s++);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t < nc) slot(acc2[t2][t], a2, hb[t], false);
      if (p >= 0 && t < nc) pairs3(p, t);
    }
  };
  auto layer3 = [&](int k3, int p) __attribute__((always_inline)) {
    const bf16x8 a3 = take(s++);
    const int buf = k3 & 1;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (2 * k3 + 1 >= kQT2) b3[buf][t][2] = b3[buf][t][3] = 0u;  // row tile 7 does not exist
      const bf16x8 b = __builtin_bit_cast(bf16x8, u32x4{b3[buf][t][0], b3[buf][t][1], b3[buf][t][2], b3[buf][t][3]});
      if (t < nc) slot(acc3[t], a3, b, k3 == 0);
      if (p >= 0 && t < nc) pairs3(p, t);
    }
  };
  static_assert(kQT2 == 7 && kQK3 == 4, "the tail below is written for 7 row tiles, 4 layer-3 k-blocks");
  layer2(0, -1);
  layer2(1, 0);
  layer2(2, 1);
  layer3(0, 2);
  layer2(3, -1);
  layer2(4, 3);
  layer3(1, 4);
  layer2(5, -1);
  layer2(6, 5);
  layer3(2, 6);
  layer3(3, -1);
  qnet_gather_q(acc3, q);
}

// qnet_mlp on nc (1..4, wave-uniform) column tiles: one instance per count. Every call site inlines
// all four, so the kernels keep one or two call sites (a pass loop), not one per pass. A weight
// fragment feeds nc MFMAs, so the fewer the column tiles the less of a fragment's load latency its
// MFMAs cover: the ring deepens as nc falls (D(nc) fragments in flight, D the full forward's; the
// fewer accumulators of a narrow instance leave the registers for it).
template <int D, class Src>
__device__ __forceinline__ void qnet_mlp_nc(const Src& src, bf16x8 xb0, bf16x8 xb1, float (&q)[8], int nc) {
  switch (nc) {
    case 1:
      qnet_mlp<4 * D, 1>(src, xb0, xb1, q);
      break;
    case 2:
      qnet_mlp<2 * D, 2>(src, xb0, xb1, q);
      break;
    case 3:
      qnet_mlp<D + D / 2, 3>(src, xb0, xb1, q);
      break;
    default:
      qnet_mlp<D, 4>(src, xb0, xb1, q);
  }
}

// the forward of a net in LDS
__device__ __forceinline__ void qnet_mlp_swp(const uint8_t* net, bf16x8 xb0, bf16x8 xb1, float (&q)[8]) {
  qnet_mlp<kQLdsAhead>(qnet_lds(net), xb0, xb1, q);
}
__device__ __forceinline__ void qnet_mlp_swp_nc(const uint8_t* net, bf16x8 xb0, bf16x8 xb1, float (&q)[8], int nc) {
  qnet_mlp_nc<kQLdsAhead>(qnet_lds(net), xb0, xb1, q, nc);
}

// Q-values of this lane's env (rows 0..7) from the block's f32 observation tile in LDS.
// row0 = tile row of this wave's lane 0. swap = the opponent's view state[5:] + state[:5]
// (scripts/main.py:199, human_player.py:40-41). Every lane of the wave must call it.
__device__ __forceinline__ void qnet_forward_swp(const uint8_t* net, const float* tile, int row0,
                                                 bool swap, float (&q)[8]) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  qnet_mlp_swp(net, qnet_input(tile + (row0 + r) * kObs, swap, h),
               qnet_input(tile + (row0 + 32 + r) * kObs, swap, h), q);
}

// ---------------------------------------------------------------------------- 32x32 forward
// The all-32x32x16 forward (rounds 1-3), kept for the config-5 instances without a net opponent
// (qnet_rollout_ws_kernel<0 / 1>). There the Q-net wave shares its SIMD's vector issue with an
// env wave that needs as much of it, and an MFMA holds the issue 8 cycles whatever its shape
// (MI355X_MICROARCH.md): 132 MFMAs per forward hold it 1,056 cycles, the 16x16 forward's 226 hold
// it 1,808. A/B at 2^20 envs, same process (profiles/r03/ab/qnet_16x16_ab_r03af.txt): ego-only
// 49.6 us/step with this forward, 53.2 with the 16x16 one; self-play 91.5 against 85.4.
// Its packed layout follows the 16x16 fragments in the same buffer (mg_qnet_pack writes both):
// W1 [204 x 24], W2 [104 x 232], W3 [9 x 136] bf16 rows (strides conflict-free for
// ds_read_b128), transposed as above with hidden units on the 32 rows of a tile; registers
// 8s..8s+7 of lane half h of a 32x32 accumulator hold rows 16s + 8(j>>2) + 4h + (j&3), and W2 / W3
// store each 16-column block in that k order, so an accumulator feeds the next MFMA directly.
constexpr int kQ32H1 = 224, kQ32H2 = 128;  // padded 200, 100
constexpr int kQ32S1 = 24, kQ32S2 = 232, kQ32S3 = 136;  // row strides (bf16)
// Stored rows: only up to the last row that can be non-zero plus one zero row (W1: units
// 0..202 + zero row 203; W2: 0..102 + zero row 103; W3: outputs 0..7 + zero row 8). A lane
// whose tile row lies past them reads the zero row instead (q32row*).
constexpr int kQ32R1 = 204, kQ32R2 = 104, kQ32R3 = 9;                    // stored rows per matrix
constexpr int kQ32OffW2 = kQ32R1 * kQ32S1 * 2;                           // ds_read_b128 lane group hits
constexpr int kQ32OffW3 = kQ32OffW2 + kQ32R2 * kQ32S2 * 2;                 // 16 distinct 4-bank slots
constexpr int kQ32NetBytes = kQ32OffW3 + kQ32R3 * kQ32S3 * 2;              // 60,496 B
static_assert(kQ32OffW2 % 16 == 0 && kQ32OffW3 % 16 == 0 && kQ32NetBytes % 16 == 0 && kQNetBytes % 16 == 0,
              "packed Q-net sections must stay 16-byte aligned");

__device__ __forceinline__ int q32row1(int m) { return m < kQ32R1 ? m : kQ32R1 - 1; }
__device__ __forceinline__ int q32row2(int m) { return m < kQ32R2 ? m : kQ32R2 - 1; }
__device__ __forceinline__ int q32row3(int m) { return m < kQ32R3 ? m : kQ32R3 - 1; }

// hardware k (0..15) within a 16-block -> hidden unit within that block (see above)
__host__ __device__ constexpr int q32_krow(int kk) {
  return 8 * ((kk & 7) >> 2) + 4 * (kk >> 3) + (kk & 3);
}

__device__ __forceinline__ bf16x8 relu_bf16(const f32x16& c, int s) {
  const int b = 8 * s;
  return __builtin_bit_cast(bf16x8, u32x4{relu_pair(c[b], c[b + 1]), relu_pair(c[b + 2], c[b + 3]),
                                          relu_pair(c[b + 4], c[b + 5]), relu_pair(c[b + 6], c[b + 7])});
}

// Packs fp32 torch Linear weights (row-major [out][in]) and biases into the kernel layout.
__global__ void qnet32_pack_kernel(const float* w1, const float* b1, const float* w2, const float* b2,
                                 const float* w3, const float* b3, int in_dim, int out_dim,
                                 uint8_t* packed) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  __bf16* pw1 = reinterpret_cast<__bf16*>(packed);
  __bf16* pw2 = reinterpret_cast<__bf16*>(packed + kQ32OffW2);
  __bf16* pw3 = reinterpret_cast<__bf16*>(packed + kQ32OffW3);
  // part p (0 hi, 1 mid, 2 lo) of the three-way bf16 split of b (hi + mid + lo == b)
  auto part = [](float b, int p) {
    const float hi = static_cast<float>(static_cast<__bf16>(b));
    const float r = b - hi;
    const float mid = static_cast<float>(static_cast<__bf16>(r));
    return p == 0 ? hi : p == 1 ? mid : r - mid;
  };
  if (e < kQ32R1 * kQ32S1) {  // W1[m][k]: natural k order (the input features), then b1's parts
    const int m = e / kQ32S1, k = e % kQ32S1;
    float v = 0.f;
    if (m < kQH1Real && k < in_dim) v = w1[m * in_dim + k];
    else if (m < kQH1Real && k >= kQBiasIn && k < kQBiasIn + 3) v = part(b1[m], k - kQBiasIn);
    else if (m >= kQOne1 && m < kQOne1 + 3 && k == kQBiasIn) v = 1.f;  // hidden-1 units = 1.0
    pw1[e] = static_cast<__bf16>(v);
    return;
  }
  e -= kQ32R1 * kQ32S1;
  if (e < kQ32R2 * kQ32S2) {  // W2[m][c]: columns in the accumulator's k order, then b2's parts
    const int m = e / kQ32S2, c = e % kQ32S2;
    const int src = 16 * (c / 16) + q32_krow(c % 16);
    float v = 0.f;
    if (c < kQ32H1) {
      if (m < kQH2Real && src < kQH1Real) v = w2[m * kQH1Real + src];
      else if (m < kQH2Real && src >= kQOne1 && src < kQOne1 + 3) v = part(b2[m], src - kQOne1);
      else if (m >= kQOne2 && m < kQOne2 + 3 && src == kQOne1) v = 1.f;  // hidden-2 units = 1.0
    }
    pw2[e] = static_cast<__bf16>(v);
    return;
  }
  e -= kQ32R2 * kQ32S2;
  if (e < kQ32R3 * kQ32S3) {  // W3[m][c], then b3's parts
    const int m = e / kQ32S3, c = e % kQ32S3;
    const int src = 16 * (c / 16) + q32_krow(c % 16);
    float v = 0.f;
    if (m < out_dim && c < kQ32H2) {
      if (src < kQH2Real) v = w3[m * kQH2Real + src];
      else if (src >= kQOne2 && src < kQOne2 + 3) v = part(b3[m], src - kQOne2);
    }
    pw3[e] = static_cast<__bf16>(v);
  }
}

// Rows 0-3 of the env of lane 32t + r sit in registers 0-3 of lane half 0 of column tile t,
// rows 4-7 in lane half 1. One v_permlane32_swap per register pair (gfx950) exchanges tile 0's
// upper half with tile 1's lower half: afterwards register j of the first operand holds row j and
// of the second row 4 + j of the lane's own env, in both lane halves (the ds_bpermute round trip
// plus selects it replaces sat between the forward's last MFMA and the argmax).
__device__ __forceinline__ void qnet32_gather_q(const f32x16& acc3_0, const f32x16& acc3_1, int h,
                                              float (&q)[8]) {
  (void)h;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // operands into locals first and the result read as one 64-bit value: hipcc (ROCm 7.2)
    // passed element 0 for every j when the builtin's arguments were subscripts, and returned
    // the first result for both subscripts of its 2-vector
    const float a = acc3_0[j], b = acc3_1[j];
    const uint32_t x = __builtin_bit_cast(uint32_t, a), y = __builtin_bit_cast(uint32_t, b);
    const uint64_t sw = __builtin_bit_cast(uint64_t, __builtin_amdgcn_permlane32_swap(x, y, false, false));
    q[j] = __builtin_bit_cast(float, static_cast<uint32_t>(sw));
    q[4 + j] = __builtin_bit_cast(float, static_cast<uint32_t>(sw >> 32));
  }
}

__device__ __forceinline__ void qnet32_mlp(const uint8_t* net, bf16x8 xb0, bf16x8 xb1, float (&q)[8]) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int z = opaque_zero();
  const __bf16* W1 = reinterpret_cast<const __bf16*>(net) + z;
  const __bf16* W2 = reinterpret_cast<const __bf16*>(net + kQ32OffW2) + z;
  const __bf16* W3 = reinterpret_cast<const __bf16*>(net + kQ32OffW3) + z;
  f32x16 acc2a[4] = {}, acc2b[4] = {};
  const f32x16 zero = {};
  auto layer1 = [&](int mt, f32x16& c0, f32x16& c1) {
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(W1 + q32row1(32 * mt + r) * kQ32S1 + 8 * h);
    c0 = mfma32(a1, xb0, zero);
    c1 = mfma32(a1, xb1, zero);
  };
  f32x16 c0, c1;
  layer1(0, c0, c1);
  // hb[f]: f = 0, 1 -> column tile 0 k-steps 0, 1; f = 2, 3 -> column tile 1
  bf16x8 hb[4] = {relu_bf16(c0, 0), relu_bf16(c0, 1), relu_bf16(c1, 0), relu_bf16(c1, 1)};
  auto w2frag = [&](int mt, int j) {
    return *reinterpret_cast<const bf16x8*>(W2 + q32row2(32 * (j >> 1) + r) * kQ32S2 + 16 * (2 * mt + (j & 1)) + 8 * h);
  };
  // one hidden tile: its layer 2, with the next tile's layer 1 + ReLU folded in when `more`
  // (a constant at every call site). nk: 16-unit k-blocks of the tile that hold real units --
  // the last tile's second block (units 208-223) is all padding, so it is skipped.
  auto tile_step = [&](int mt, bool more, int nk) __attribute__((always_inline)) {
    bf16x8 a2n = w2frag(mt, 0);
    if (more) layer1(mt + 1, c0, c1);
    uint32_t nx[16];  // next tile's packed ReLU pairs, built between this tile's MFMAs
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m2 = j >> 1, sk = j & 1;
      if (sk >= nk) continue;
      // one fragment ahead: the next load is in flight under this pair of MFMAs
      const bf16x8 a2 = a2n;
      const int jn = nk == 2 ? j + 1 : j + 2;
      if (jn < 8) a2n = w2frag(mt, jn);
      __builtin_amdgcn_sched_barrier(0);
      acc2a[m2] = mfma32(a2, hb[sk], acc2a[m2]);
      acc2b[m2] = mfma32(a2, hb[2 + sk], acc2b[m2]);
      if (more) {
#pragma unroll
        for (int pp = 2 * j; pp < 2 * j + 2; ++pp) {
          const int f = pp >> 2, b = 8 * (f & 1) + 2 * (pp & 3);
          const f32x16& c = f < 2 ? c0 : c1;
          nx[pp] = relu_pair(c[b], c[b + 1]);
        }
      }
    }
    if (more) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
        hb[f] = __builtin_bit_cast(bf16x8, u32x4{nx[4 * f], nx[4 * f + 1], nx[4 * f + 2], nx[4 * f + 3]});
    }
  };
  constexpr int kLast = kQ32H1 / 32 - 1;
  static_assert(16 * (2 * kLast + 1) >= kQH1Real && 32 * kLast < kQH1Real,
                "only the last hidden tile's second k-block is padding");
#pragma unroll
  for (int mt = 0; mt < kLast; ++mt) tile_step(mt, true, 2);
  // The last hidden tile (its k-block 0 only) interleaved with layer 3, over the k-blocks holding
  // real units (96..111 carries units 100..102 = 1.0 too; 112..127 is padding). acc2a/b[m2] are
  // final once the tile's pair m2 has issued, so layer 3's k-blocks 2 m2 and 2 m2 + 1 -- their
  // ReLU and MFMAs, in the same order as before -- follow pair m2 + 1 instead of the whole tile:
  // the tile's MFMAs had no vector work beside them and layer 3 is mostly vector work. W2 and W3
  // fragments one ahead.
  f32x16 acc3_0 = {}, acc3_1 = {};
  auto w3frag = [&](int kb) { return *reinterpret_cast<const bf16x8*>(W3 + q32row3(r) * kQ32S3 + 16 * kb + 8 * h); };
  constexpr int kK3 = (kQH2Real + 15) / 16;
  static_assert(kK3 == 7 && kQ32H2 / 32 == 4, "layer 3 k-blocks 2 m2, 2 m2 + 1 follow layer-2 row tile m2");
  bf16x8 a3n = w3frag(0);
  auto layer3 = [&](int m2) __attribute__((always_inline)) {
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const int kb = 2 * m2 + sk;
      if (kb >= kK3) continue;
      const bf16x8 a3 = a3n;
      if (kb + 1 < kK3) a3n = w3frag(kb + 1);
      acc3_0 = mfma32(a3, relu_bf16(acc2a[m2], sk), acc3_0);
      acc3_1 = mfma32(a3, relu_bf16(acc2b[m2], sk), acc3_1);
    }
  };
  bf16x8 a2n = w2frag(kLast, 0);
#pragma unroll
  for (int m2 = 0; m2 < kQ32H2 / 32; ++m2) {
    const bf16x8 a2 = a2n;
    if (m2 + 1 < kQ32H2 / 32) a2n = w2frag(kLast, 2 * (m2 + 1));
    __builtin_amdgcn_sched_barrier(0);
    acc2a[m2] = mfma32(a2, hb[0], acc2a[m2]);
    acc2b[m2] = mfma32(a2, hb[2], acc2b[m2]);
    if (m2 > 0) layer3(m2 - 1);
  }
  layer3(kQ32H2 / 32 - 1);
  qnet32_gather_q(acc3_0, acc3_1, h, q);
}

// the 32x32 forward of a net whose 32x32 layout is in LDS, from the block's observation tile
__device__ __forceinline__ void qnet32_forward(const uint8_t* net32, const float* tile, int row0, bool swap,
                                               float (&q)[8]) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  qnet32_mlp(net32, qnet_input(tile + (row0 + r) * kObs, swap, h), qnet_input(tile + (row0 + 32 + r) * kObs, swap, h), q);
}

// mg_qnet_fragments: the packed layout is fragment-major itself since ABI 19, so the "fragment
// copy" the h-DQN opponent is read from is a plain copy (kept so the ABI-18 callers run unchanged)
__global__ __launch_bounds__(64) void qnet_fragments_kernel(const uint8_t* packed, uint8_t* frags) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i < kQNetBytes / 16) reinterpret_cast<u32x4*>(frags)[i] = reinterpret_cast<const u32x4*>(packed)[i];
}

// This lane's rank among the set lanes of a ballot (lanes below it whose bit is set).
__device__ __forceinline__ int lane_rank(uint64_t m) {
  return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}

// 16-env column tiles of a forward over n (1..64) compacted items
__device__ __forceinline__ int col_tiles(int n) { return (n + 15) >> 4; }

__device__ __forceinline__ int argmax_first(const float (&q)[8], int out_dim) {
  int best = 0;
  float v = q[0];
#pragma unroll
  for (int j = 1; j < 8; ++j)
    if (j < out_dim && q[j] > v) {
      v = q[j];
      best = j;
    }
  return best;
}

// Standalone forward for tests / evaluation: q[i][0..7] for x[i][0..in_dim-1], staged in LDS as
// 16-float rows (swap, in_dim 10 only: the features in the order state[5:] + state[:5]).
__global__ __launch_bounds__(kBlock) void qnet_forward_kernel(const uint8_t* net, const float* x,
                                                              int in_dim, int swap, float* qout,
                                                              int64_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kQNetBytes];
  __shared__ __attribute__((aligned(16))) float tile[kBlock * 16];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock;
  qnet_to_lds(net, lds_net);
  for (int j = threadIdx.x; j < kBlock * 16; j += kBlock) {
    const int64_t i = base + (j >> 4);
    const int k = j & 15;
    const int src = swap ? (k + kObs / 2) % kObs : k;
    tile[j] = (i < n && k < in_dim) ? x[i * in_dim + src]
              : (k >= kQBiasIn && k < kQBiasIn + 3) ? 1.f : 0.f;
  }
  __syncthreads();
  float q[8];
  {
    const int lane = threadIdx.x & 63, row0 = (threadIdx.x >> 6) * 64;
    qnet_mlp_swp(lds_net, qnet_input_wide(tile + (row0 + (lane & 31)) * 16, lane >> 5),
                 qnet_input_wide(tile + (row0 + 32 + (lane & 31)) * 16, lane >> 5), q);
  }
  const int64_t i = base + threadIdx.x;
  if (i < n) {
#pragma unroll
    for (int j = 0; j < 8; ++j) qout[i * 8 + j] = q[j];
  }
}

// may_finish_next's constants (below)
struct FinishBound {
  float smin, smax, g;  // min / max of action_dict, the MPC's speed gain per step
  float lat, lon;       // collision reach before the step: lateral |y1 - y2| and longitudinal |x1 - x2|
                        // (finish_bound, from veh_w / veh_h / R / dT and the speeds: 5.75 / 9 by default)
};

// may_finish_next's constants for these params (host). Collision after the step needs
// trunc(y1) - trunc(y2) <= veh_w, so y1 - y2 < veh_w + 1, and |x1 - x2| < veh_h + 1 (the pygame
// Rect truncation of vehicle_box). A step moves a car by dl <= dT vmax along its arc, vmax =
// max(start_vel, action speeds) + 0.5 (a speed only moves toward an action's target), and so its
// lateral y by at most dl |sin theta|; where y1 - y2 < lat the ego's 1 - cos theta < lat / R, so
// |sin theta| < sqrt(2 lat / R) + dl / R over the step. lat = veh_w + 1 + max(0.75, 2 dl sin + 0.25):
// the default params' 0.75 (5.75) stands unless the geometry needs more. The longitudinal reach of
// the speeds is added at run time (rel in may_finish_next).
inline FinishBound finish_bound(const mg_params& P) {
  double smin = P.action_speed[0], smax = smin;
  for (int a = 1; a < MG_NUM_ACTIONS; ++a) {
    smin = std::min(smin, P.action_speed[a]);
    smax = std::max(smax, P.action_speed[a]);
  }
  const double vmax = std::max(smax, P.start_vel) + 0.5;
  const double dl = P.dT * vmax;
  double lat = P.veh_w + 1.75;
  for (int it = 0; it < 4; ++it) {  // lat appears in its own bound: a few fixed-point passes
    const double sn = std::sqrt(2.0 * lat / P.R) + dl / P.R;
    lat = P.veh_w + 1.0 + std::max(0.75, 2.0 * dl * sn + 0.25);
  }
  // rounded outward by a margin: the bound only has to contain every speed a step reaches
  return FinishBound{static_cast<float>(smin) - 0.5f, static_cast<float>(smax) + 0.5f,
                     static_cast<float>(P.dT * P.qp_z0 / P.qp_nz) * 1.01f, static_cast<float>(lat),
                     static_cast<float>(P.veh_h + 1)};
}
struct QRollout {
  mg_params P;
  Reset0 R0;
  mg_state S;
  mg_traj T;
  mg_stats St;
  const uint8_t* net;
  const uint8_t* opp_net;   // OPP 3: the opponent's own net (main.py's Strategy_OP "L1")
  uint64_t seed;
  uint64_t first_step;
  uint64_t greedy_thr;      // greedy iff u32 draw < greedy_thr (2^32: always)
  uint64_t opp_greedy_thr;
  int64_t env_offset;
  int64_t n;
  int32_t num_steps;
  int32_t out_dim;
  uint32_t flags;
  FinishBound fin;  // may_finish_next's constants
};

// Whether env e's next step can end its episode, for ANY pair of actions (a conservative superset of
// env_step's done, tests/test_may_finish.py): main.py:221 logs eval_net(state)[action] of an
// episode's last step whatever branch chose the action, so the config-5 kernels evaluate the net for
// these envs even where the ego explores. From the state a step acts on (o: its fp32 observation;
// every margin below is >= 0.25 m, far above the fp32 rounding of o):
//   timeout   the step count reaches timeout_steps (env_clock);
//   arrival   a car can pass END_POINT within the step and that ends the episode (the other car
//             already won, or both arrive): p' = p + dT v' with v' between v and the action's target
//             speed, so END_POINT - p < dT max(v, smax) + 0.5;
//   collision the boxes can overlap afterwards. Laterally trunc(y1) - trunc(y2) <= veh_w needs
//             y1 - y2 < veh_w + 1 (y1 >= y2 on the two arcs), and a step moves each y by at most
//             |sin theta| dT v' (< 0.17 m there by default); B.lat (finish_bound) covers both.
//             Longitudinally |t1 - t2| <= veh_h needs |x1 - x2| < veh_h + 1 (B.lon), and a
//             step changes x1 - x2 by at most dT |v1' - v2'| (+ 0.2 % for the arc): the MPC moves each
//             speed by g (s - v), g = dT z0 / z'n = 1/15 (mpc_acc), so |v1' - v2'| <= |v1 - v2| +
//             g (max(smax, v1, v2) - min(smin, v1, v2)).
// Flags ~2.2 % of env-steps in uniform random play (tests/test_may_finish.py).
MG_HD bool may_finish_next(const mg_params& P, const Env& e, const obs_t (&o)[kObs], const FinishBound& B) {
  if (static_cast<int32_t>(e.steps) + 1 >= P.timeout_steps) return true;
  const float dt = static_cast<float>(P.dT);
  const bool ego = o[3] < dt * fmaxf(o[4], B.smax) + 0.5f;  // o[3] = END_POINT - p1, o[4] = v1
  const bool opp = o[8] < dt * fmaxf(o[9], B.smax) + 0.5f;  // o[8] = END_POINT - p2, o[9] = v2
  const bool arrive = e.winner == 1 ? opp : (e.winner == 2 ? ego : (ego && opp));
  const float spread = fmaxf(B.smax, fmaxf(o[4], o[9])) - fminf(B.smin, fminf(o[4], o[9]));
  const float rel = dt * (fabsf(o[2]) + B.g * spread) + 0.5f;  // o[2] = v2 - v1
  const bool coll = -o[1] < B.lat && fabsf(o[0]) < B.lon + rel;  // o[1] = y2 - y1, o[0] = x2 - x1
  return arrive || coll;
}

// The need bits of env gi's step `step` for the config-5 Q-net waves (opponent modes 2 / 3): bit 0
// the ego's forward (its greedy draw, or may_finish_next while statistics are kept), bit 1 the
// opponent's (its greedy draw). u: the step's Philox words (qnet_policy_step_n's stream).
__device__ __forceinline__ uint8_t qnet_need_bits(const QRollout& R, const uint4& u, bool live, const Env& e,
                                                  const obs_t (&o)[kObs]) {
  if (!live) return 0;
  const bool fin = R.St.rec != nullptr && (R.flags & MG_AUTORESET) && may_finish_next(R.P, e, o, R.fin);
  return static_cast<uint8_t>(((static_cast<uint64_t>(u.x) < R.greedy_thr || fin) ? 1 : 0) |
                              (static_cast<uint64_t>(u.z) < R.opp_greedy_thr ? 2 : 0) | (fin ? 4 : 0));
}

// Where the Q-net waves find them: OPP 2 reads both bits from greedy[1][j]; OPP 3 (round 5, the
// waves split by net) gives each net's waves a byte of their own -- greedy[0][j] the ego's (bit 0
// need, bit 1 may finish), greedy[1][j] the opponent's (bit 0 its greedy draw, bit 1 may finish) --
// which those waves then overwrite with the greedy actions, so no byte is shared between waves.
template <int OPP>
__device__ __forceinline__ void qnet_put_need(uint8_t* g0, uint8_t* g1, uint8_t b) {
  if constexpr (OPP == 3) {
    const uint8_t fin = static_cast<uint8_t>((b >> 1) & 2);
    *g0 = static_cast<uint8_t>((b & 1) | fin);
    *g1 = static_cast<uint8_t>(((b >> 1) & 1) | fin);
  } else {
    *g1 = b;
  }
}

__device__ __forceinline__ uint4 qnet_draws(const QRollout& R, int64_t i, uint64_t step) {
  const uint64_t gi = static_cast<uint64_t>(R.env_offset + i);
  return philox4x32_10(make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32),
                                  static_cast<uint32_t>(step), static_cast<uint32_t>(step >> 32)),
                       static_cast<uint32_t>(R.seed), static_cast<uint32_t>(R.seed >> 32));
}


// One epsilon-greedy step (main.py:99-112) of the N envs i0 + 64 j of one env-wave lane given their
// greedy actions, stepped in lockstep. Draws (ABI 20), Philox4x32-10 keyed by seed:
//  * OPP 0 / 1 (no net opponent): two draws per step, so one call serves two steps -- step k takes
//    words (x, y) of call (gi, k div 2) when k is even and (z, w) when k is odd (kept from the even
//    step in `keep`, or computed when a launch starts on an odd step). The first word is the ego's
//    explore draw; the second its random action floor(5 w / 2^32), or with the uniform opponent the
//    pair x = floor(25 w / 2^32), a1 = x div 5, a2 = x mod 5 (one word, as the random-policy stream).
//  * OPP 2 / 3: call (gi, k) per step: u.x the ego's explore draw, u.y its random action, u.z the
//    opponent's explore draw, u.w its random action.
// Envs past n (live[j] false) are stepped too but never stored. A greedy action outside 0..4 (a
// net with out_dim > 5) gets env_step's KeyError semantics (env_step_lockstep).
// qrow: the tile row of env i0 (rows of envs i0 + 64 j follow 64 rows apart), where the Q-net wave
// left eval_net(state)[0..4] of the state the step acts on: a finishing env logs q[a1] (main.py:221).
template <int OPP, int N, bool CHECKED>
__device__ __forceinline__ void qnet_policy_step_n(const QRollout& R, Env (&e)[N], StepOut (&r)[N],
                                                   int64_t i0, const bool (&live)[N], int t,
                                                   const int (&greedy1)[N], const int (&greedy2)[N],
                                                   bool (&won)[N], const float* qrow, uint2 (&keep)[N],
                                                   double (&pend)[N], uint4 (&un)[N], uint8_t* need0,
                                                   uint8_t* need1) {
  const uint64_t step = R.first_step + t;
  int a1[N], a2[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint64_t gi = static_cast<uint64_t>(R.env_offset + i0 + 64 * j);
    if constexpr (OPP < 2) {
      uint32_t ex, pick;
      if ((step & 1) == 0 || t == 0) {  // wave-uniform: a fresh call feeds this step and the next
        const uint4 u = philox4x32_10(
            make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32),
                       static_cast<uint32_t>(step >> 1), static_cast<uint32_t>(step >> 33)),
            static_cast<uint32_t>(R.seed), static_cast<uint32_t>(R.seed >> 32));
        keep[j] = make_uint2(u.z, u.w);
        ex = (step & 1) ? u.z : u.x;
        pick = (step & 1) ? u.w : u.y;
      } else {
        ex = keep[j].x;
        pick = keep[j].y;
      }
      const bool greedy = static_cast<uint64_t>(ex) < R.greedy_thr;
      if constexpr (OPP == 1) {  // (random a1, uniform a2) from one 25-way draw
        const uint32_t x = static_cast<uint32_t>((static_cast<uint64_t>(pick) * 25u) >> 32);
        const int b1 = static_cast<int>((x * 13u) >> 6);  // x div 5 for x < 25
        a1[j] = greedy ? greedy1[j] : b1;
        a2[j] = static_cast<int>(x) - 5 * b1;
      } else {
        a1[j] = greedy ? greedy1[j] : action_from_u32(pick);
        a2[j] = MG_ACTION_NONE;
      }
    } else {
      const uint4 u = un[j];  // drawn one phase ahead, with the need bits the Q-net waves compacted by
      a1[j] = (static_cast<uint64_t>(u.x) < R.greedy_thr) ? greedy1[j] : action_from_u32(u.y);
      a2[j] = (static_cast<uint64_t>(u.z) < R.opp_greedy_thr) ? greedy2[j] : action_from_u32(u.w);
    }
  }
  env_step_lockstep<N, CHECKED>(R.P, e, a1, a2, r);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    won[j] = false;
    if (!live[j]) continue;
    const int64_t i = i0 + 64 * j;
    const int64_t row = static_cast<int64_t>(t) * R.n + i;
    if (R.T.rew)
      st_out(reinterpret_cast<f32x2*>(R.T.rew) + row,
             f32x2{static_cast<float>(r[j].r1), static_cast<float>(r[j].r2)});
    store_step_bytes(R.T, row, a1[j], a2[j], r[j].done, r[j].coll);
    won[j] = e[j].winner == 1;
    // the Q value the scripts log for a finished episode (q_eval_value, main.py:221); a1 in 0..4
    // here (a bad action leaves done false)
    if (after_step_nowait(R.P, e[j], r[j], R.St, R.T.final_obs ? R.T.final_obs + row * kObs : nullptr, i,
                          (R.flags & MG_AUTORESET) != 0, pend[j], &R.R0))
      add_q_eval_nowait(R.St, i, qrow[64 * j * kObs + a1[j]]);
  }
  if constexpr (OPP >= 2) {  // the next step's draws and need bits, for Q(X, t + 1)
    if (t + 1 < R.num_steps) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        un[j] = qnet_draws(R, i0 + 64 * j, step + 1);
        qnet_put_need<OPP>(need0 + 64 * j, need1 + 64 * j, qnet_need_bits(R, un[j], live[j], e[j], r[j].o));
      }
    }
  }
}

// Observation of env i (or zeros past n) into its fp32 tile row; returns live.
__device__ __forceinline__ bool qnet_load_env(const QRollout& R, int64_t i, Env& e, float* row) {
  double o[kObs];
  const bool live = i < R.n;
  if (live) {
    e = load_env(R.S, i);
    double x1, y1, x2, y2;
    lon2coord(R.P, e.p1, true, x1, y1);
    lon2coord(R.P, e.p2, false, x2, y2);
    observe(R.P, e.p1, e.v1, e.p2, e.v2, x1, y1, x2, y2, o);
  } else {  // a defined state for the lockstep step, which also steps envs past n (never stored)
    e.p1 = e.p2 = R.P.start_point;
    e.v1 = e.v2 = R.P.start_vel;
    e.ret1 = e.ret2 = 0.0;
    e.steps = 0;
    e.winner = 0;
    e.done = false;
#pragma unroll
    for (int k = 0; k < kObs; ++k) o[k] = 0.0;
  }
  float2* t2 = reinterpret_cast<float2*>(row);
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k)
    t2[k] = make_float2(static_cast<float>(o[2 * k]), static_cast<float>(o[2 * k + 1]));
  return live;
}


// The same T steps with the waves specialised: waves 0-3 run only the Q-net (matrix cores +
// ReLU), waves 4-7 only the fp64 env step, so each SIMD pairs a matrix-heavy wave with a
// vector-heavy one (waves w and w + 4 share a SIMD). The block's 512 envs are two groups
// of 256, pipelined over 2T + 1 barrier-separated phases:
//   Q(A,0) | Q(B,0) + step(A,0) | Q(A,1) + step(B,0) | ... | step(B,T-1)
// Greedy actions go to the env waves through LDS; the new observations come back through the
// tile rows. Each env-wave lane holds the two envs (one per group) it steps.
// OPP 3 (main.py's default Strategy_OP "L1", :161-168: the opponent is another trained DQN)
// keeps a second net in LDS: with the 16x16 layouts (2 x 59,392 B, ABI 19) the two nets, the
// 1,024-env tile and the greedy bytes take 161,792 B, so it runs ILP 2 like the others (the
// 32x32 layouts, 2 x 60,496 B, did not fit and ran ILP 1 on 512-env blocks: 1 % slower).
// The items a Q-net wave runs itself out of a list of n (round 5): all of them, or 192 (three full
// forwards) when 1..16 remain past those, which then run on the env wave of the same index.
__device__ __forceinline__ int qws_own_items(int n) { return n > 192 && n <= 192 + 16 ? 192 : n; }
__device__ __forceinline__ void qws_publish_tail(int (&qt)[4], int p, int nq, int nn, int nf) {
  if ((threadIdx.x & 63) == 0) {
    qt[1] = nq;
    qt[2] = nn;
    qt[3] = nf;
    __hip_atomic_store(&qt[0], p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}
__device__ __forceinline__ void qws_wait(const int* flag, int p) {
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != p) __builtin_amdgcn_s_sleep(1);
}

template <int OPP>
constexpr int qws_ilp() { return kQWsIlp; }
template <int OPP>
constexpr int qws_envs() { return 2 * 64 * kQWsEnvWaves * qws_ilp<OPP>(); }

// CHECKED: a greedy action may fall outside action_dict (a net with out_dim > 5): the lockstep step
// carries the KeyError selects. Every other launch takes CHECKED = false (-2 % on the ego-only
// leg, r03i; the self-play and other-net instances showed no gain and keep the checked step).
template <int OPP, bool CHECKED>
__global__ __launch_bounds__(kQWsThreads, kQWsWavesPerSimd) void qnet_rollout_ws_kernel(const QRollout R) {
  constexpr int kIlp = qws_ilp<OPP>();
  constexpr int kEnvs = qws_envs<OPP>();  // envs per block
  constexpr int kHalf = kEnvs / 2;        // envs per group
  constexpr int kTiles = kHalf / 256;     // 64-env tiles each Q-net wave computes per phase
  constexpr int kEnvWaves = kQWsEnvWaves;
  static_assert(kTiles >= 1 && kHalf == 64 * kEnvWaves * kIlp && kHalf % 256 == 0,
                "group = 4 Q-net waves x kTiles x 64 envs = env waves x ILP x 64 envs");
  // OPP 0 / 1: the 32x32 layout (second part of the packed buffer) and forward, see qnet32_mlp
  constexpr bool kNet32 = OPP < 2;
  __shared__ __attribute__((aligned(16))) uint8_t lds_net[kNet32 ? kQ32NetBytes : kQNetBytes];
  __shared__ __attribute__((aligned(16))) uint8_t lds_net2[OPP == 3 ? kQNetBytes : 16];
  __shared__ __attribute__((aligned(16))) float tile[kEnvs * kObs];
  __shared__ uint8_t greedy[2][kEnvs];
  // OPP 2 / 3 (round 5): per Q-net wave the compacted items of a phase -- OPP 2: env e of the wave's
  // 128 | 0x80 the opponent's view; OPP 3: env e of the wave's 256 (one net per wave). When a phase
  // begins the greedy bytes hold the need bits (qnet_need_bits, qnet_put_need)
  __shared__ uint8_t qlist[OPP >= 2 ? 4 : 1][OPP >= 2 ? 256 : 1];
  // OPP 2: each listed item's layer-1 B fragment halves (the view it needs), staged by the env's own
  // lane, so one forward can hold both views' items (one net) and reads its inputs lane-linearly:
  // half-major ([wave][h][item]), so the 32 lanes reading one half read 512 contiguous bytes (round 6;
  // item-major, the 32-B item stride left half of the banks idle: SQ_LDS_BANK_CONFLICT / IDX_ACTIVE
  // 0.097, valu_busy.json)
  __shared__ __attribute__((aligned(16))) u32x4 qstage[OPP == 2 ? 4 : 1][2][OPP == 2 ? 256 : 1];
  // OPP 3: phase p once opponent wave h has read every tile row an ego wave will overwrite with
  // Q-values (the may-finish rows, which it lists first)
  __shared__ int qrows_read[2];
  // OPP 2 / 3: a Q-net wave's list tail -- its items past three full forwards, when at most 16 -- runs
  // on env wave w (the same index) after that wave's step, so the Q-net waves' phase ends after three
  // forwards instead of three and a narrow fourth (whose weight stream costs half a full one). Wave w
  // publishes {phase, items it runs, list length, may-finish items} once its list (and OPP 2's staged
  // fragments) are in LDS; the phase word last, with release order.
  __shared__ int qtail[OPP >= 2 ? 4 : 1][4];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kEnvs;
  const bool qwave = wave < 4;
  const int ew = wave - 4;

  if constexpr (kNet32) {
    const f32x4* src = reinterpret_cast<const f32x4*>(R.net + kQNetBytes);
    for (int j = tid; j < kQ32NetBytes / 16; j += blockDim.x) reinterpret_cast<f32x4*>(lds_net)[j] = src[j];
  } else {
    qnet_to_lds(R.net, lds_net);
  }
  if constexpr (OPP == 3) qnet_to_lds(R.opp_net, lds_net2);
  if (tid < 2) qrows_read[tid] = -1;
  if (OPP >= 2 && tid < 4) qtail[tid][0] = -1;
  const int phases = 2 * R.num_steps + 1;
  if (qwave) {
    // Q-net waves: the barrier count matches the env waves' loop below, phase for phase
    // (roles are whole waves, so s_barrier pairs up; the two loops keep each role's live
    // registers apart -- in one loop the env state sat beside the accumulators and spilled)
    __syncthreads();
    for (int p = 0; p < phases; ++p) {
      if constexpr (OPP == 3) {
        // Only the forwards the reference evaluates (round 5; OPP 2 below for the common part), with
        // the waves split by net: waves 0-1 run the opponent's net, 2-3 the ego's, each over 256 of
        // the group's 512 envs (rows rb + e). One net per wave keeps the view uniform and gives each
        // wave ~194 items = three full 64-item forwards and a narrow one; split by env instead, each
        // wave ran both nets on ~97 items apiece (two forwards per net, the second three tiles wide).
        // An ego wave writes eval_net(state)[0..4] into the tile rows of its may-finish items only (an
        // episode can end only there, main.py:221) and only once the opponent wave of the same rows
        // has read them: that wave lists those items first and publishes the phase in
        // qrows_read[hw] after their forward; the ego wave lists them last.
        if (p < 2 * R.num_steps) {
          static_assert(kHalf == 512, "two waves per net, 256 envs each");
          const bool oppw = wave < 2;
          const int hw = wave & 1;
          const int rb = (p & 1) * kHalf + 256 * hw;
          uint8_t* gout = greedy[oppw ? 1 : 0] + rb;
          uint8_t* list = qlist[wave];
          uint64_t mn[4], mf[4];
          int nn = 0, nf = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int nb = gout[64 * k + lane];
            mn[k] = __ballot(nb & 1);
            mf[k] = __ballot((nb & 3) == 3);
            nn += __popcll(mn[k]);
            nf += __popcll(mf[k]);
          }
          int of = oppw ? 0 : nn - nf, on = oppw ? nf : 0;  // may-finish items first / last
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint64_t mo = mn[k] & ~mf[k];
            if ((mf[k] >> lane) & 1)
              list[of + lane_rank(mf[k])] = static_cast<uint8_t>(64 * k + lane);
            else if ((mo >> lane) & 1)
              list[on + lane_rank(mo)] = static_cast<uint8_t>(64 * k + lane);
            of += __popcll(mf[k]);
            on += __popcll(mo);
          }
          wave_lds_sync();
          const int nq = qws_own_items(nn);
          qws_publish_tail(qtail[wave], p, nq, nn, nf);
          if (oppw && nf == 0 && lane == 0) __hip_atomic_store(&qrows_read[hw], p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int fin0 = nn - nf;  // an ego wave's first may-finish item
          const int r = lane & 31, h = lane >> 5;
          const uint8_t* net = oppw ? lds_net2 : lds_net;
          // the tile rows of a chunk's items (column envs r and 32 + r, and this lane's result row),
          // read one chunk ahead: a forward's inputs then wait for one LDS read, not two
          auto rows_of = [&](int c, int& ra, int& rc, int& ro) __attribute__((always_inline)) {
            const int n = nn - c < 64 ? nn - c : 64;
            ra = rb + list[c + (r < n ? r : 0)];
            rc = rb + list[c + (32 + r < n ? 32 + r : 0)];
            ro = rb + list[c + (lane < n ? lane : 0)];
          };
          int ra, rc, row;
          rows_of(0, ra, rc, row);
#pragma unroll 1
          for (int c0 = 0; c0 < nq;) {
            const int cnt = nq - c0 < 64 ? nq - c0 : 64;
            auto input = [&](int j) __attribute__((always_inline)) {
              const float* rw = tile + j * kObs;
              return oppw ? qnet_input(rw, true, h) : qnet_input(rw, false, h);
            };
            const bf16x8 x0 = input(ra), x1 = input(rc);
            const int rcur = row;
            if (c0 + cnt < nq) rows_of(c0 + cnt, ra, rc, row);
            float q[8];
            qnet_mlp_swp_nc(net, x0, x1, q, col_tiles(cnt));
            if (lane < cnt) gout[rcur - rb] = static_cast<uint8_t>(argmax_first(q, R.out_dim));
            if (oppw) {  // (nf > nq: the env wave running the tail publishes it)
              if (c0 < nf && c0 + cnt >= nf && lane == 0)  // the forward has consumed its rows
                __hip_atomic_store(&qrows_read[hw], p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (c0 + cnt > fin0) {
              qws_wait(&qrows_read[hw], p);
              if (lane < cnt && c0 + lane >= fin0) {
                float* qr = tile + rcur * kObs;
                reinterpret_cast<f32x2*>(qr)[0] = f32x2{q[0], q[1]};
                reinterpret_cast<f32x2*>(qr)[1] = f32x2{q[2], q[3]};
                qr[4] = q[4];
              }
            }
            wave_lds_sync();
            c0 += cnt;
          }
        }
        __syncthreads();
        continue;
      }
      if constexpr (OPP == 2) {
        // Only the forwards the reference evaluates (round 5): choose_action runs the net on its
        // greedy branch only (main.py:105-107), and :221 evaluates it on an episode's last step.
        // The wave's 128 envs of the group are compacted by their need bits into one list, the
        // opponent's items (swapped view) first, and each view's items run through the forward 64
        // at a time on col_tiles(count) column tiles. The ego's q[0..4] go into the env's tile row
        // for q_eval, after every read of that row (the opponent items come first).
        if (p < 2 * R.num_steps) {
          static_assert(kTiles == 2, "the list holds the wave's two 64-env tiles");
          const int gb = (p & 1) * kHalf;
          auto row_of = [&](int e) __attribute__((always_inline)) { return gb + (4 * ((e >> 6) & 1) + wave) * 64 + (e & 63); };
          uint8_t* list = qlist[wave];
          const int nb0 = greedy[1][row_of(lane)], nb1 = greedy[1][row_of(64 + lane)];
          const uint64_t mo0 = __ballot(nb0 & 2), mo1 = __ballot(nb1 & 2);
          const uint64_t me0 = __ballot(nb0 & 1), me1 = __ballot(nb1 & 1);
          const int Lo0 = __popcll(mo0), Lo = Lo0 + __popcll(mo1);
          const int Le0 = __popcll(me0), Ln = Lo + Le0 + __popcll(me1);
          if (nb0 & 2) list[lane_rank(mo0)] = static_cast<uint8_t>(0x80 | lane);
          if (nb1 & 2) list[Lo0 + lane_rank(mo1)] = static_cast<uint8_t>(0x80 | 64 | lane);
          if (nb0 & 1) list[Lo + lane_rank(me0)] = static_cast<uint8_t>(lane);
          if (nb1 & 1) list[Lo + Le0 + lane_rank(me1)] = static_cast<uint8_t>(64 | lane);
          {
            // the same net for both views: stage every item's fragments from its env's lane (both
            // views of the row from one read), then run the whole list 64 items per forward
            auto stage = [&](int row, int nb, int po, int pe) __attribute__((always_inline)) {
              float f[kObs];
#pragma unroll
              for (int k = 0; k < kObs / 2; ++k) {
                const f32x2 t2 = reinterpret_cast<const f32x2*>(tile + row * kObs)[k];
                f[2 * k] = t2[0];
                f[2 * k + 1] = t2[1];
              }
              auto pk = [](float a, float b) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2)); };
              if (nb & 2) {  // the opponent's view state[5:] + state[:5] (main.py:199)
                qstage[wave][0][po] = u32x4{pk(f[5], f[6]), pk(f[7], f[8]), pk(f[9], f[0]), pk(f[1], f[2])};
                qstage[wave][1][po] = u32x4{pk(f[3], f[4]), 0u, 0x3F800000u, 0x3F803F80u};
              }
              if (nb & 1) {
                qstage[wave][0][pe] = u32x4{pk(f[0], f[1]), pk(f[2], f[3]), pk(f[4], f[5]), pk(f[6], f[7])};
                qstage[wave][1][pe] = u32x4{pk(f[8], f[9]), 0u, 0x3F800000u, 0x3F803F80u};
              }
            };
            stage(row_of(lane), nb0, lane_rank(mo0), Lo + lane_rank(me0));
            stage(row_of(64 + lane), nb1, Lo0 + lane_rank(mo1), Lo + Le0 + lane_rank(me1));
          }
          wave_lds_sync();
          const int nq = qws_own_items(Ln);
          qws_publish_tail(qtail[wave], p, nq, Ln, 0);
          const int r = lane & 31, h = lane >> 5;
#pragma unroll 1
          for (int c0 = 0; c0 < nq;) {
            // staged fragments, any mix of views (a view chosen per lane by selects on the features
            // cost +35 % per launch, r05f q1 / q2)
            const int cnt = nq - c0 < 64 ? nq - c0 : 64;
            auto input = [&](int it) __attribute__((always_inline)) {
              return __builtin_bit_cast(bf16x8, qstage[wave][h][c0 + (it < cnt ? it : 0)]);
            };
            const int e_out = list[c0 + (lane < cnt ? lane : 0)];  // read ahead: its wait hides under the forward
            float q[8];
            qnet_mlp_swp_nc(lds_net, input(r), input(32 + r), q, col_tiles(cnt));
            if (lane < cnt) {
              const int e = e_out;
              const int row = row_of(e);
              const uint8_t a = static_cast<uint8_t>(argmax_first(q, R.out_dim));
              if (e & 0x80) {
                greedy[1][row] = a;
              } else {
                greedy[0][row] = a;
                // eval_net(state)[0..4] into the row the env wave reads at an episode end (main.py:221)
                float* qr = tile + row * kObs;
                reinterpret_cast<f32x2*>(qr)[0] = f32x2{q[0], q[1]};
                reinterpret_cast<f32x2*>(qr)[1] = f32x2{q[2], q[3]};
                qr[4] = q[4];
              }
            }
            wave_lds_sync();
            c0 += cnt;
          }
        }
        __syncthreads();
        continue;
      }
      if (p < 2 * R.num_steps) {
#pragma unroll 1
        for (int tt = 0; tt < kTiles; ++tt) {
          const int row0 = (p & 1) * kHalf + (4 * tt + wave) * 64;
          float q[8];
          if constexpr (OPP >= 2) {  // the opponent's view state[5:] + state[:5] (main.py:199)
            qnet_forward_swp(OPP == 3 ? lds_net2 : lds_net, tile, row0, true, q);
            greedy[1][row0 + lane] = static_cast<uint8_t>(argmax_first(q, R.out_dim));
          }
          if constexpr (kNet32)
            qnet32_forward(lds_net, tile, row0, false, q);
          else
            qnet_forward_swp(lds_net, tile, row0, false, q);
          greedy[0][row0 + lane] = static_cast<uint8_t>(argmax_first(q, R.out_dim));
          // eval_net(state)[0..4] into the env's tile row, whose observation both forwards have
          // read (the MFMA chain behind q waits for every read): the env wave steps the env in the
          // next phase and logs q[action] when the episode ends (main.py:221), before it writes
          // the next observation into the row
          float* qr = tile + (row0 + lane) * kObs;
          reinterpret_cast<f32x2*>(qr)[0] = f32x2{q[0], q[1]};
          reinterpret_cast<f32x2*>(qr)[1] = f32x2{q[2], q[3]};
          qr[4] = q[4];
        }
      }
      __syncthreads();
    }
    return;
  }
  // env lane: envs lbase + 64 j + lane (j < kIlp) of group 0 (e0) and of group 1 (e1)
  const int lbase = ew * 64 * kIlp;
  Env e0[kIlp], e1[kIlp];
  StepOut r[kIlp];
  bool live0[kIlp], live1[kIlp];
  uint2 keep0[kIlp], keep1[kIlp];  // OPP 0 / 1: the odd step's two draw words (qnet_policy_step_n)
  double pend0[kIlp], pend1[kIlp];  // main.py's pending values (pend_load, after_step_nowait)
  uint4 un0[kIlp], un1[kIlp];       // OPP 2 / 3: each env's draws of its next step (one phase ahead)
#pragma unroll
  for (int j = 0; j < kIlp; ++j) {
    const int la = lbase + 64 * j + lane, lb = kHalf + la;
    live0[j] = qnet_load_env(R, base + la, e0[j], tile + la * kObs);
    live1[j] = qnet_load_env(R, base + lb, e1[j], tile + lb * kObs);
    pend0[j] = live0[j] ? pend_load(R.St, base + la, e0[j]) : 0.0;
    pend1[j] = live1[j] ? pend_load(R.St, base + lb, e1[j]) : 0.0;
    if constexpr (OPP >= 2) {  // step 0's draws and need bits (the observation as the tile row holds it)
      obs_t o0[kObs], o1[kObs];
#pragma unroll
      for (int k = 0; k < kObs; ++k) {
        o0[k] = tile[la * kObs + k];
        o1[k] = tile[lb * kObs + k];
      }
      un0[j] = qnet_draws(R, base + la, R.first_step);
      un1[j] = qnet_draws(R, base + lb, R.first_step);
      qnet_put_need<OPP>(&greedy[0][la], &greedy[1][la], qnet_need_bits(R, un0[j], live0[j], e0[j], o0));
      qnet_put_need<OPP>(&greedy[0][lb], &greedy[1][lb], qnet_need_bits(R, un1[j], live1[j], e1[j], o1));
    }
#pragma unroll
    for (int k = 0; k < kObs; ++k) r[j].o[k] = 0.0;
  }
  __syncthreads();
  for (int p = 0; p < phases; ++p) {
    if (p > 0) {
      const int g = (p - 1) & 1, t = (p - 1) >> 1;
      const int local0 = g * kHalf + lbase;
      int greedy1[kIlp], greedy2[kIlp];
#pragma unroll
      for (int j = 0; j < kIlp; ++j) {
        greedy1[j] = greedy[0][local0 + 64 * j + lane];
        greedy2[j] = OPP >= 2 ? greedy[1][local0 + 64 * j + lane] : 0;
      }
      bool won[kIlp];
      // wave-uniform branch: each group's envs stay in named registers
      const float* qrow = tile + (local0 + lane) * kObs;
      uint8_t* need0 = &greedy[0][local0 + lane];
      uint8_t* need1 = &greedy[1][local0 + lane];
      if (g == 0)
        qnet_policy_step_n<OPP, kIlp, CHECKED>(R, e0, r, base + local0 + lane, live0, t, greedy1, greedy2, won, qrow,
                                               keep0, pend0, un0, need0, need1);
      else
        qnet_policy_step_n<OPP, kIlp, CHECKED>(R, e1, r, base + local0 + lane, live1, t, greedy1, greedy2, won, qrow,
                                               keep1, pend1, un1, need0, need1);
      const int64_t wbase = base + local0;
#pragma unroll
      for (int j = 0; j < kIlp; ++j) {
        const int64_t rem = R.n - (wbase + 64 * j);
        store_won_mask(R.T.won_mask, won[j], t, R.n, wbase + 64 * j,
                       rem <= 0 ? 0 : (rem < 64 ? static_cast<int>(rem) : 64));
      }
      const int64_t wrem = R.n - wbase;
      const int wrows = wrem <= 0 ? 0 : (wrem < 64 * kIlp ? static_cast<int>(wrem) : 64 * kIlp);
      wave_store_obs_n<kIlp>(tile + local0 * kObs, r,
                             R.T.obs ? R.T.obs + (static_cast<int64_t>(t) * R.n + wbase) * kObs : nullptr,
                             wrows);
    }
    if constexpr (OPP >= 2) {
      // Q-net wave ew's list tail for Q(group p & 1, step p / 2), as that wave would run it (qtail)
      if (p < 2 * R.num_steps) {
        qws_wait(&qtail[ew][0], p);
        const int nq = qtail[ew][1], nn = qtail[ew][2];
        if (nn > nq) {
          const int cnt = nn - nq;  // 1..16: one column tile
          const uint8_t* list = qlist[ew];
          const int r32 = lane & 31, h = lane >> 5;
          const int it = nq + (r32 < cnt ? r32 : 0), io = nq + (lane < cnt ? lane : 0);
          float q[8];
          if constexpr (OPP == 3) {
            const bool oppw = ew < 2;
            const int hw = ew & 1, nf = qtail[ew][3];
            const int rb = (p & 1) * kHalf + 256 * hw;
            const float* rw = tile + (rb + list[it]) * kObs;
            const int row = rb + list[io];
            const bf16x8 x = oppw ? qnet_input(rw, true, h) : qnet_input(rw, false, h);
            qnet_mlp<2 * kQLdsAhead, 1>(qnet_lds(oppw ? lds_net2 : lds_net), x, x, q);
            if (lane < cnt) greedy[oppw ? 1 : 0][row] = static_cast<uint8_t>(argmax_first(q, R.out_dim));
            if (oppw) {
              if (nf > nq && lane == 0) __hip_atomic_store(&qrows_read[hw], p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (nn - nf < nn) {  // may-finish items, listed last
              qws_wait(&qrows_read[hw], p);
              if (lane < cnt && io >= nn - nf) {
                float* qr = tile + row * kObs;
                reinterpret_cast<f32x2*>(qr)[0] = f32x2{q[0], q[1]};
                reinterpret_cast<f32x2*>(qr)[1] = f32x2{q[2], q[3]};
                qr[4] = q[4];
              }
            }
          } else {
            const bf16x8 x = __builtin_bit_cast(bf16x8, qstage[ew][h][it]);
            qnet_mlp<2 * kQLdsAhead, 1>(qnet_lds(lds_net), x, x, q);
            if (lane < cnt) {
              const int e = list[io];
              const int row = (p & 1) * kHalf + (4 * ((e >> 6) & 1) + ew) * 64 + (e & 63);
              const uint8_t a = static_cast<uint8_t>(argmax_first(q, R.out_dim));
              if (e & 0x80) {
                greedy[1][row] = a;
              } else {
                greedy[0][row] = a;
                float* qr = tile + row * kObs;
                reinterpret_cast<f32x2*>(qr)[0] = f32x2{q[0], q[1]};
                reinterpret_cast<f32x2*>(qr)[1] = f32x2{q[2], q[3]};
                qr[4] = q[4];
              }
            }
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kIlp; ++j) {
    const int la = lbase + 64 * j + lane;
    if (live0[j]) store_env(R.S, base + la, e0[j]);
    if (live1[j]) store_env(R.S, base + kHalf + la, e1[j]);
  }
}

// memory_counter += k (the fused goal ring's stores are all kept: no scan)
__global__ void counter_add_kernel(uint64_t* counter, uint64_t k) { *counter += k; }

// ============================================================================ h-DQN acting loop
// hdqn.py's inner loop (scripts/hdqn.py:280-323) in one launch: Goal_DQN's meta-net picks the
// sub-goal on every next state (:303), the lower-level Net acts on the goal state
// [goal] + state (:291-292), goal_status (:223-237) gives the intrinsic reward (:314) and ends
// the inner loop (:320-322), after which -- and after every episode end (:278-283, the outer
// loops) -- a fresh goal is chosen. Both nets live in LDS (compact packing, 2 x 60.5 KB).
//
// OPP 2 is hdqn.py's Strategy_OP "selfplay" (:262-264, upper_op = upper, lower_op = lower): the
// same two nets also choose the opponent's goal on the swapped state at every outer-loop
// iteration (:285) and its action on [goal_op] + swapped state (:299-300), two more forwards per
// phase on the Q-net waves.
// Per env-step k (global step index) the Philox4x32-10 streams are
//   A = Philox(counter (gi, k)):            x ego explore draw, y ego random action,
//                                           z goal explore draw, w random goal (the goal
//                                           chosen on the step's next state, :303)
//   B = Philox(counter (gi ^ 2^63, k)):     x, y the same for a fresh goal (after a goal was
//                                           reached or the episode ended, :283), z the uniform
//                                           opponent's action (opponent_mode 1)
//   C = Philox(counter (gi ^ 2^62, k)):     (OPP 2) x explore, y action of the opponent's
//                                           step, z explore, w goal of its fresh goal at k + 1
// and a launch whose env has no goal yet (goal[i] < 0) starts it with B of step first_step - 1.
// Roles as in qnet_rollout_ws_kernel: waves 0-3 run both nets (meta then lower, one 64-env tile
// each per phase), waves 4-7 the fp64 env step (one env per lane), on two groups of 256 envs
// pipelined over 2T + 2 phases: Q(A,0) | Q(B,0) + E(A,0) | ... | Q(A,T) + E(B,T-1) | Q(B,T).
// Q(X,t) finishes step t-1's goal logic (meta on its next state: the terminal observation where
// the episode ended, kept in LDS as bf16 pairs) and picks step t's action; E(X,t) steps.
struct HRollout {
  mg_params P;
  Reset0 R0;
  mg_state S;
  mg_traj T;
  mg_hdqn_traj H;
  mg_stats St;
  int8_t* goal;     // [n] in / out
  int8_t* goal_op;  // [n] in / out, the self-play opponent's goal (OPP 2)
  double* ext_acc;  // [n] in / out, extrinsic reward since the inner loop began (Goal_DQN rows)
  const uint8_t* meta;
  const uint8_t* lower;
  const uint8_t* meta_op;   // OPP 3: the opponent's own nets, fragment-major (read from L2)
  const uint8_t* lower_op;
  uint64_t seed;
  uint64_t first_step;
  uint64_t greedy_thr;
  int64_t env_offset;
  int64_t n;
  int32_t num_steps;
  int32_t num_goals;
  int32_t reset_goal;
  uint32_t flags;
  // fused goal ring (hdqn.py:316 stores every transition, so slots need no scan): rows
  // [goal, s, a, r, next_goal, s'] of transition (t, i) at (counter0 + t n + i) % capacity
  float* ring;  // [capacity, 24] or NULL
  const uint64_t* ring_counter;
  int64_t ring_capacity;
};

constexpr int kHEnvs = 512;              // envs per block: two groups of 256
constexpr int kRowGoalF = 2 * kObs + 4;  // goal ring row floats (hdqn.py:158)
constexpr int kHHalf = kHEnvs / 2;
constexpr uint8_t kHGreedy = 0xFF;       // draw byte: take the greedy choice

__device__ __forceinline__ uint8_t draw_byte(uint32_t explore, uint32_t pick, uint64_t thr, int k) {
  return static_cast<uint8_t>(static_cast<uint64_t>(explore) < thr
                                  ? kHGreedy
                                  : (static_cast<uint64_t>(pick) * static_cast<uint64_t>(k)) >> 32);
}

__device__ __forceinline__ uint4 philox_env_step(uint64_t gi, uint64_t step, uint64_t seed) {
  return philox4x32_10(make_uint4(static_cast<uint32_t>(gi), static_cast<uint32_t>(gi >> 32),
                                  static_cast<uint32_t>(step), static_cast<uint32_t>(step >> 32)),
                       static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
}

// The fresh-goal draws (explore, goal) of step k from stream B (counter gi ^ 2^63). Every opponent
// but the uniform one uses two words of B per step, so one call serves two steps (ABI 20): call
// k div 2, words (x, y) on even steps and (z, w) on odd ones; `keep` carries the odd step's pair
// from the even step (fresh: compute the call, as at a launch's first step). The uniform opponent
// also draws its action from B (word z of call k), one call per step.
template <int OPP>
__device__ __forceinline__ uint2 fresh_goal_words(uint64_t gi, uint64_t k, uint64_t seed, bool fresh, uint2& keep,
                                                  uint32_t& opp_word) {
  if constexpr (OPP == 1) {
    const uint4 u = philox_env_step(gi ^ (uint64_t{1} << 63), k, seed);
    opp_word = u.z;
    return make_uint2(u.x, u.y);
  } else {
    opp_word = 0u;
    if ((k & 1) == 0 || fresh) {
      const uint4 u = philox_env_step(gi ^ (uint64_t{1} << 63), k >> 1, seed);
      keep = make_uint2(u.z, u.w);
      return (k & 1) ? keep : make_uint2(u.x, u.y);
    }
    return keep;
  }
}

// lower-net input of one env: goal state [goal] + state (hdqn.py:291), features 0..10, zero at
// 11..12 and the bias inputs 1.0 at 13..15; swap: [goal] + state[5:] + state[:5] (the
// opponent's goal state, :299)
__device__ __forceinline__ bf16x8 qnet_input_goal(const float* row, int goal, int h, bool swap = false) {
  float v[kObs];
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k) {
    const f32x2 t = reinterpret_cast<const f32x2*>(row)[k];
    // swapped view state[5:] + state[:5]: pair (4, 5) straddles the halves, so each element
    // takes its own destination (element 5 -> v[0], element 4 -> v[9])
    const int d0 = swap ? (2 * k + kObs / 2) % kObs : 2 * k;
    const int d1 = swap ? (2 * k + 1 + kObs / 2) % kObs : 2 * k + 1;
    v[d0] = t[0];
    v[d1] = t[1];
  }
  auto pk = [](float a, float b) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2)); };
  const u32x4 w = h ? u32x4{pk(v[7], v[8]), pk(v[9], 0.f), 0x3F800000u, 0x3F803F80u}
                    : u32x4{pk(static_cast<float>(goal), v[0]), pk(v[1], v[2]), pk(v[3], v[4]), pk(v[5], v[6])};
  return __builtin_bit_cast(bf16x8, w);
}

// meta-net input of one env from its bf16-pair side row (the terminal observation)
__device__ __forceinline__ bf16x8 qnet_input_pairs(const uint32_t* side, int h) {
  return __builtin_bit_cast(bf16x8, h ? u32x4{side[4], 0u, 0x3F800000u, 0x3F803F80u}
                                      : u32x4{side[0], side[1], side[2], side[3]});
}

template <int OPP>
__global__ __launch_bounds__(512, 2) void hdqn_rollout_kernel(const HRollout R) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_meta[kQNetBytes];
  __shared__ __attribute__((aligned(16))) uint8_t lds_lower[kQNetBytes];
  __shared__ __attribute__((aligned(16))) float tile[kHEnvs * kObs];    // s' (reset obs where done)
  __shared__ __attribute__((aligned(16))) uint32_t side[kHEnvs * 5];    // terminal obs, bf16 pairs
  __shared__ uint8_t b_act[kHEnvs], b_goal[kHEnvs], b_done[kHEnvs], b_st_old[kHEnvs],
      b_st_new[kHEnvs], b_dg[kHEnvs], b_df[kHEnvs], b_g2[kHEnvs];
  // OPP 2 / 3: the opponent's greedy action, current goal and fresh-goal draw
  constexpr bool kOpNets = OPP >= 2;  // the opponent acts through h-DQN nets
  __shared__ uint8_t b_aop[kOpNets ? kHEnvs : 1], b_gop[kOpNets ? kHEnvs : 1], b_dfo[kOpNets ? kHEnvs : 1];
  // the opponent meta-net's compacted items per Q-net wave and their goals (round 5)
  __shared__ uint8_t b_olist[kOpNets ? 4 : 1][64], b_gos[kOpNets ? kHEnvs : 1];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kHEnvs;
  const int T = R.num_steps;
  const int phases = 2 * T + 2;
  {
    const f32x4* s1 = reinterpret_cast<const f32x4*>(R.meta);
    const f32x4* s2 = reinterpret_cast<const f32x4*>(R.lower);
    f32x4* d1 = reinterpret_cast<f32x4*>(lds_meta);
    f32x4* d2 = reinterpret_cast<f32x4*>(lds_lower);
    for (int j = tid; j < kQNetBytes / 16; j += blockDim.x) {
      d1[j] = s1[j];
      d2[j] = s2[j];
    }
  }
  if (wave < 4) {
    // ---------------------------------------------------------------- the two nets
    __syncthreads();
    const int r = lane & 31, h = lane >> 5;
    for (int p = 0; p < phases; ++p) {
      const int g = p & 1, t = p >> 1;
      const int row0 = g * kHHalf + 64 * wave;  // this wave's 64 envs: rows row0 + lane
      const int j = row0 + lane;
      const int64_t i = base + j;
      const bool live = i < R.n;
      // This env's bytes for the phase, read together before the meta forward and held across it
      // (round 5: read where used, after the forward, each put an LDS round trip on the Q-net
      // waves' chain -- the goal logic took ~1.1 k cycles per phase, tools/clk_segments.py)
      const int goal_prev = static_cast<int8_t>(b_goal[j]);
      const int dg = b_dg[j], df = b_df[j], st_new = b_st_new[j], st_old = b_st_old[j];
      const bool done = t > 0 && b_done[j] != 0;
      int gop_prev = 0, dfo = 0;
      if constexpr (kOpNets) {
        gop_prev = static_cast<int8_t>(b_gop[j]);
        dfo = b_dfo[j];
      }
      int goal_t;
      const bool need_meta = t > 0 || __ballot(live && goal_prev < 0) != 0;
      int gstar = 0;
      float qe = 0.f;  // meta_eval_net(terminal state)[goal chosen on it], logged at an episode end (:330)
      if (need_meta) {  // meta-net on the next state of step t - 1 (on s_0 for a launch's first goals)
        // both sources read at once, the terminal observation's bf16 pairs chosen where the episode
        // ended (one LDS round trip, not the done byte's and then the row's)
        const bool d0 = t > 0 && b_done[row0 + r], d1 = t > 0 && b_done[row0 + 32 + r];
        const bf16x8 p0 = qnet_input_pairs(side + (row0 + r) * 5, h), p1 = qnet_input_pairs(side + (row0 + 32 + r) * 5, h);
        const bf16x8 o0 = qnet_input(tile + (row0 + r) * kObs, false, h);
        const bf16x8 o1 = qnet_input(tile + (row0 + 32 + r) * kObs, false, h);
        const bf16x8 x0 = d0 ? p0 : o0, x1 = d1 ? p1 : o1;
        // the bytes above arrive with the inputs (one wait), not after the forward
        asm volatile("" ::"v"(dg), "v"(df), "v"(st_new), "v"(st_old), "v"(gop_prev), "v"(dfo));
        float q[8];
        qnet_mlp_swp(lds_meta, x0, x1, q);
        gstar = argmax_first(q, R.num_goals);
        const int g2 = dg == kHGreedy ? gstar : dg;
#pragma unroll
        for (int k = 0; k < 8; ++k) qe = k == g2 ? q[k] : qe;
      }
      bool brk = false;  // step t - 1 left the inner loop (:322): a new outer iteration starts
      if (t > 0) {  // hdqn.py:303-322 for step t - 1
        const int goal2 = dg == kHGreedy ? gstar : dg;
        brk = done || goal2 == st_new;
        goal_t = done ? (df == kHGreedy ? R.reset_goal : df) : (brk ? (df == kHGreedy ? gstar : df) : goal2);
        if (live) {
          const int64_t row = static_cast<int64_t>(t - 1) * R.n + i;
          if (R.H.next_goal) st_out(R.H.next_goal + row, static_cast<float>(goal2));
          if (R.H.reward) st_out(R.H.reward + row, goal2 == st_old ? 1.0f : 0.0f);
        }
        b_g2[j] = static_cast<uint8_t>(goal2);  // for the fused ring row of step t - 1
        // the episode's q_eval (hdqn.py:330): the env wave recorded the episode in E(X, t - 1); this
        // lane is the only writer of the field, so no-return atomics keep the adds in step order
        if (done && live) add_q_eval_nowait(R.St, i, static_cast<double>(qe));
      } else {
        goal_t = goal_prev >= 0 ? goal_prev : (df == kHGreedy ? gstar : df);
      }
      int gop_t = 0;
      if constexpr (kOpNets) {  // upper_op.choose_goal(swapped state) at a new outer iteration (:285)
        const bool fresh_op = t > 0 ? brk : gop_prev < 0;
        // Only where the reference evaluates it (round 5): at a new outer iteration, on the greedy
        // branch (:86-92) -- about a quarter of the envs. The wave's items are compacted into one
        // forward on 32 envs (two column tiles) when they fit, else the full 64; the other passes
        // run at three quarters or more and stay uncompacted (a forward's weight stream costs as
        // much as two column tiles, so a narrower pass than two tiles' saving does not pay).
        const bool need_o = live && fresh_op && dfo == kHGreedy;
        const uint64_t mo = __ballot(need_o);
        int gop_star = 0;
        if (mo != 0) {  // on the state acted on at step t (reset obs after an end)
          const int L = __popcll(mo);
          uint8_t* list = b_olist[wave];
          if (need_o) list[lane_rank(mo)] = static_cast<uint8_t>(lane);
          wave_lds_sync();
          const int ea = list[r < L ? r : 0], ec = list[32 + r < L ? 32 + r : 0], eo = list[lane < L ? lane : 0];
          float q[8];
          const bf16x8 x0 = qnet_input(tile + (row0 + ea) * kObs, true, h);
          const bf16x8 x1 = qnet_input(tile + (row0 + ec) * kObs, true, h);
          if constexpr (OPP == 3) {  // the opponent's own Goal_DQN (:267)
            if (L <= 32)
              qnet_mlp<2 * kQGlobalAhead, 2>(qnet_global(R.meta_op), x0, x1, q);
            else
              qnet_mlp<kQGlobalAhead>(qnet_global(R.meta_op), x0, x1, q);
          } else {
            if (L <= 32)
              qnet_mlp<2 * kQLdsAhead, 2>(qnet_lds(lds_meta), x0, x1, q);
            else
              qnet_mlp_swp(lds_meta, x0, x1, q);
          }
          if (lane < L) b_gos[row0 + eo] = static_cast<uint8_t>(argmax_first(q, R.num_goals));
          wave_lds_sync();
          gop_star = b_gos[j];  // this env's item where need_o
        }
        gop_t = fresh_op ? (dfo == kHGreedy ? gop_star : dfo) : gop_prev;
      }
      if (t < T) {
        b_goal[j] = static_cast<uint8_t>(goal_t);
        if (live && R.H.goal) st_out(R.H.goal + static_cast<int64_t>(t) * R.n + i, static_cast<float>(goal_t));
        if constexpr (kOpNets) {
          b_gop[j] = static_cast<uint8_t>(gop_t);
          if (live && R.H.goal_op) st_out(R.H.goal_op + static_cast<int64_t>(t) * R.n + i, static_cast<float>(gop_t));
        }
        wave_lds_sync();  // the wave's goals are in LDS before the lanes read their column envs'
        const bf16x8 xe0 = qnet_input_goal(tile + (row0 + r) * kObs, b_goal[row0 + r], h);
        const bf16x8 xe1 = qnet_input_goal(tile + (row0 + 32 + r) * kObs, b_goal[row0 + 32 + r], h);
        // the opponent's inputs too, before the ego's forward (held across it)
        bf16x8 xo0 = xe0, xo1 = xe1;
        if constexpr (kOpNets) {
          xo0 = qnet_input_goal(tile + (row0 + r) * kObs, b_gop[row0 + r], h, true);
          xo1 = qnet_input_goal(tile + (row0 + 32 + r) * kObs, b_gop[row0 + 32 + r], h, true);
        }
        float q[8];
        qnet_mlp_swp(lds_lower, xe0, xe1, q);
        b_act[j] = static_cast<uint8_t>(argmax_first(q, MG_NUM_ACTIONS));
        if constexpr (kOpNets) {  // lower_op.choose_action([goal_op] + swapped state) (:299-300)
          float qo[8];
          const bf16x8 x0 = xo0, x1 = xo1;
          if constexpr (OPP == 3)
            qnet_mlp<kQGlobalAhead>(qnet_global(R.lower_op), x0, x1, qo);  // the opponent's own HDQN (:268)
          else
            qnet_mlp_swp(lds_lower, x0, x1, qo);
          b_aop[j] = static_cast<uint8_t>(argmax_first(qo, MG_NUM_ACTIONS));
        }
      } else if (live) {
        R.goal[i] = static_cast<int8_t>(goal_t);  // the next launch's starting goal
        if constexpr (kOpNets) R.goal_op[i] = static_cast<int8_t>(gop_t);
      }
      __syncthreads();
    }
    return;
  }
  // ------------------------------------------------------------------ the env step
  const int ew = wave - 4;
  Env e[2];
  bool live[2];
  double pend[2] = {0.0, 0.0};  // main.py's pending values (pend_load, after_step_nowait)
  int stc[2];  // goal_status of each group's current state, from its fp64 dx1 and v2
  // the fused ring row of each group's last step, completed once the Q-net waves have chosen
  // its next goal: s, s' (terminal where done), goal, action
  float ps[2][kObs], ps2[2][kObs];
  int pgoal[2], pact[2];
  // Goal_DQN's memory (hdqn.py:286, :311-313, :322, :325): the extrinsic reward since each env's
  // inner loop began, and at each step whether that loop ended (known once Q(X, t + 1) has chosen
  // the step's next goal, so it is emitted together with the ring row of the step)
  // kept whenever the caller holds the running sums (ext_acc), so turning ext_reward / no_break
  // on in a later launch continues the loops already in flight correctly
  const bool outer = R.ext_acc != nullptr;
  double acc[2] = {0.0, 0.0};
  uint2 kb[2] = {make_uint2(0u, 0u), make_uint2(0u, 0u)};  // each group's odd-step fresh-goal words
  auto finish_outer = [&](int g, int t, double& ac) __attribute__((always_inline)) {
    const int j = g * kHHalf + 64 * ew + lane;
    const int64_t i = base + j;
    const int64_t wbase = base + g * kHHalf + 64 * ew;
    const bool lv = i < R.n;
    const bool brk = b_done[j] != 0 || b_g2[j] == b_st_new[j];
    if (R.H.ext_reward && lv) st_out(R.H.ext_reward + static_cast<int64_t>(t) * R.n + i, static_cast<float>(ac));
    if (R.H.no_break) {
      const uint64_t m = __ballot(lv && !brk);
      if (lane == 0 && wbase < R.n) st_out(R.H.no_break + static_cast<int64_t>(t) * ((R.n + 63) >> 6) + (wbase >> 6), m);
    }
    if (brk) ac = 0.0;  // :286 extrinsic_reward = 0 for the next outer iteration
  };
  const bool ring = R.ring != nullptr;
  const uint64_t c0 = ring ? *R.ring_counter : 0;
  const int64_t total = static_cast<int64_t>(T) * R.n;
  auto write_row = [&](int g, int t, const float (&s0)[kObs], const float (&s1)[kObs], int pg,
                       int pa) __attribute__((always_inline)) {
    const int j = g * kHHalf + 64 * ew + lane;
    const int64_t i = base + j;
    const int64_t k = static_cast<int64_t>(t) * R.n + i;  // transition index within the launch
    if (!ring || i >= R.n || k < total - R.ring_capacity) return;  // the newest capacity rows only
    const int goal2 = b_g2[j];
    const int st_old = b_st_old[j];
    float* row = R.ring + static_cast<int64_t>((c0 + static_cast<uint64_t>(k)) %
                                               static_cast<uint64_t>(R.ring_capacity)) * kRowGoalF;
    f32x4 v[6];
    float f[kRowGoalF];
    f[0] = static_cast<float>(pg);
#pragma unroll
    for (int q = 0; q < kObs; ++q) f[1 + q] = s0[q];
    f[11] = static_cast<float>(pa);
    f[12] = goal2 == st_old ? 1.0f : 0.0f;
    f[13] = static_cast<float>(goal2);
#pragma unroll
    for (int q = 0; q < kObs; ++q) f[14 + q] = s1[q];
#pragma unroll
    for (int q = 0; q < 6; ++q) v[q] = f32x4{f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]};
#pragma unroll
    for (int q = 0; q < 6; ++q) st_out(reinterpret_cast<f32x4*>(row) + q, v[q]);
  };
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int j = g * kHHalf + 64 * ew + lane;
    const int64_t i = base + j;
    live[g] = i < R.n;
    double o[kObs];
    if (live[g]) {
      e[g] = load_env(R.S, i);
      pend[g] = pend_load(R.St, i, e[g]);
      double x1, y1, x2, y2;
      lon2coord(R.P, e[g].p1, true, x1, y1);
      lon2coord(R.P, e[g].p2, false, x2, y2);
      observe(R.P, e[g].p1, e[g].v1, e[g].p2, e[g].v2, x1, y1, x2, y2, o);
    } else {  // a defined state, stepped but never stored
      e[g].p1 = e[g].p2 = R.P.start_point;
      e[g].v1 = e[g].v2 = R.P.start_vel;
      e[g].ret1 = e[g].ret2 = 0.0;
      e[g].steps = 0;
      e[g].winner = 0;
      e[g].done = false;
#pragma unroll
      for (int k = 0; k < kObs; ++k) o[k] = 0.0;
    }
    stc[g] = goal_status(o[0], o[9]);
    float2* t2 = reinterpret_cast<float2*>(tile + j * kObs);
#pragma unroll
    for (int k = 0; k < kObs / 2; ++k) t2[k] = make_float2(static_cast<float>(o[2 * k]), static_cast<float>(o[2 * k + 1]));
    const uint64_t gi = static_cast<uint64_t>(R.env_offset + i);
    uint2 unused_keep;
    uint32_t unused_word;
    const uint2 fb = fresh_goal_words<OPP>(gi, R.first_step - 1, R.seed, true, unused_keep, unused_word);
    b_df[j] = draw_byte(fb.x, fb.y, R.greedy_thr, R.num_goals);
    b_goal[j] = live[g] ? static_cast<uint8_t>(R.goal[i]) : 0;
    if (outer && live[g]) acc[g] = R.ext_acc[i];
    if constexpr (kOpNets) {
      const uint4 fc = philox_env_step(gi ^ (uint64_t{1} << 62), R.first_step - 1, R.seed);
      b_dfo[j] = draw_byte(fc.z, fc.w, R.greedy_thr, R.num_goals);
      b_gop[j] = live[g] ? static_cast<uint8_t>(R.goal_op[i]) : 0;
    }
    b_done[j] = 0;
  }
  __syncthreads();
  for (int p = 0; p < phases; ++p) {
    if (p > 0 && ((p - 1) >> 1) < T) {
      const int g = (p - 1) & 1, t = (p - 1) >> 1;
      const int j = g * kHHalf + 64 * ew + lane;
      const int64_t i = base + j;
      const int64_t wbase = base + g * kHHalf + 64 * ew;
      const uint64_t gi = static_cast<uint64_t>(R.env_offset + i), k = R.first_step + t;
      const uint4 ua = philox_env_step(gi, k, R.seed);
      uint32_t opp_word;
      const uint2 ub = g == 0 ? fresh_goal_words<OPP>(gi, k, R.seed, t == 0, kb[0], opp_word)
                              : fresh_goal_words<OPP>(gi, k, R.seed, t == 0, kb[1], opp_word);
      const int a1 = static_cast<uint64_t>(ua.x) < R.greedy_thr ? static_cast<int>(b_act[j]) : action_from_u32(ua.y);
      int a2 = OPP == 1 ? action_from_u32(opp_word) : MG_ACTION_NONE;
      uint4 uc = make_uint4(0u, 0u, 0u, 0u);
      if constexpr (kOpNets) {  // the self-play opponent's epsilon-greedy action (:300)
        uc = philox_env_step(gi ^ (uint64_t{1} << 62), k, R.seed);
        a2 = static_cast<uint64_t>(uc.x) < R.greedy_thr ? static_cast<int>(b_aop[j]) : action_from_u32(uc.y);
      }
      if (t > 0) {  // step t - 1's next goal is in LDS now (Q(X, t)); wave-uniform branch per group
        if (g == 0)
          write_row(0, t - 1, ps[0], ps2[0], pgoal[0], pact[0]);
        else
          write_row(1, t - 1, ps[1], ps2[1], pgoal[1], pact[1]);
        if (outer) {
          if (g == 0)
            finish_outer(0, t - 1, acc[0]);
          else
            finish_outer(1, t - 1, acc[1]);
        }
      }
      auto step = [&](Env& ev, bool lv, float (&s0)[kObs], float (&s1)[kObs], int& pg, int& pa, double& ac,
                      int& st, double& pd) __attribute__((always_inline)) {
        StepOut rv;  // per step: the state acted on is the env's tile row, so no observation is carried
        b_st_old[j] = static_cast<uint8_t>(st);  // status of the state acted on (:314)
        if (ring) {
          const f32x2* trow = reinterpret_cast<const f32x2*>(tile + j * kObs);
#pragma unroll
          for (int q = 0; q < kObs / 2; ++q) {
            const f32x2 v = trow[q];
            s0[2 * q] = v[0];
            s0[2 * q + 1] = v[1];
          }
          pg = b_goal[j];
          pa = a1;
        }
        // every action here is in action_dict: the lower nets' argmax runs over the first
        // NUM_ACTIONS outputs, the random draws are 0..4, so the step needs no KeyError path
        env_step<false>(R.P, ev, a1, a2, rv);
        ac += rv.r1;  // :311-313 extrinsic_reward += reward
        if (ring) {
#pragma unroll
          for (int q = 0; q < kObs; ++q) s1[q] = static_cast<float>(rv.o[q]);  // terminal where done
        }
        const int64_t row = static_cast<int64_t>(t) * R.n + i;
        if (lv) {
          if (R.T.rew) st_out(reinterpret_cast<f32x2*>(R.T.rew) + row, f32x2{static_cast<float>(rv.r1), static_cast<float>(rv.r2)});
          store_step_bytes(R.T, row, a1, a2, rv.done, rv.coll);
        }
        b_done[j] = rv.done ? 1 : 0;
        st = goal_status(rv.dx1, ev.v2);  // of the next state (:322), terminal where done
        b_st_new[j] = static_cast<uint8_t>(st);
        b_dg[j] = draw_byte(ua.z, ua.w, R.greedy_thr, R.num_goals);
        b_df[j] = draw_byte(ub.x, ub.y, R.greedy_thr, R.num_goals);
        if constexpr (kOpNets) b_dfo[j] = draw_byte(uc.z, uc.w, R.greedy_thr, R.num_goals);
        const bool won = lv && ev.winner == 1;
        const int64_t rem = R.n - wbase;
        store_won_mask(R.T.won_mask, won, t, R.n, wbase, rem <= 0 ? 0 : (rem < 64 ? static_cast<int>(rem) : 64));
        if (lv && (R.flags & MG_AUTORESET) && rv.done) {
          uint32_t* sd = side + j * 5;  // the terminal observation for the meta-net
#pragma unroll
          for (int q2 = 0; q2 < kObs / 2; ++q2)
            sd[q2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                                                      f32x2{static_cast<float>(rv.o[2 * q2]), static_cast<float>(rv.o[2 * q2 + 1])}, bf16x2));
          after_step_nowait(R.P, ev, rv, R.St, R.T.final_obs ? R.T.final_obs + row * kObs : nullptr, i, true, pd,
                            &R.R0);
          st = goal_status(rv.dx1, ev.v2);  // the reset state the next step acts on
        } else if (lv) {
          after_step_nowait(R.P, ev, rv, R.St, nullptr, i, false, pd, &R.R0);  // the first arrival, if any
        }
        const int64_t wrem = R.n - wbase;
        wave_store_obs(tile + (g * kHHalf + 64 * ew) * kObs, rv.o,
                       R.T.obs ? R.T.obs + (static_cast<int64_t>(t) * R.n + wbase) * kObs : nullptr,
                       wrem <= 0 ? 0 : (wrem < 64 ? static_cast<int>(wrem) : 64));
      };
      if (g == 0)
        step(e[0], live[0], ps[0], ps2[0], pgoal[0], pact[0], acc[0], stc[0], pend[0]);
      else
        step(e[1], live[1], ps[1], ps2[1], pgoal[1], pact[1], acc[1], stc[1], pend[1]);
    }
    __syncthreads();
  }
  // both groups' last rows: Q(A,T) and Q(B,T) chose their next goals in the last two phases
  write_row(0, T - 1, ps[0], ps2[0], pgoal[0], pact[0]);
  write_row(1, T - 1, ps[1], ps2[1], pgoal[1], pact[1]);
  if (outer) {
    finish_outer(0, T - 1, acc[0]);
    finish_outer(1, T - 1, acc[1]);
#pragma unroll
    for (int g = 0; g < 2; ++g)
      if (live[g]) R.ext_acc[base + g * kHHalf + 64 * ew + lane] = acc[g];
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
    if (live[g]) store_env(R.S, base + g * kHHalf + 64 * ew + lane, e[g]);
}

__global__ __launch_bounds__(kBlock) void reset_kernel(const mg_params P, const mg_state S,
                                                       const uint8_t* mask, const mg_outputs O,
                                                       int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  if (mask && !mask[i]) return;
  S.p1[i] = P.start_point;
  S.v1[i] = P.start_vel;
  S.p2[i] = P.start_point;
  S.v2[i] = P.start_vel;
  S.ret1[i] = 0.0;
  S.ret2[i] = 0.0;
  S.tf[i] = 0u;
  if (O.obs || O.rec64) {
    double o[kObs];
    reset_obs(P, o);
    if (O.obs) {
#pragma unroll
      for (int k = 0; k < kObs; ++k) O.obs[i * kObs + k] = static_cast<float>(o[k]);
    }
    if (O.rec64) {
      mg_rec64* rec = O.rec64 + i;
#pragma unroll
      for (int k = 0; k < kObs; ++k) rec->obs[k] = o[k];
      rec->rew[0] = rec->rew[1] = 0.0;
      rec->acc[0] = rec->acc[1] = 0.0;
      rec->pos[0] = rec->pos[1] = P.start_point;
      rec->vel[0] = rec->vel[1] = P.start_vel;
      rec->ret[0] = rec->ret[1] = 0.0;
      rec->tf = 0u;
      rec->status = 0u;
    }
  }
}

__global__ __launch_bounds__(kBlock) void observe_kernel(const mg_params P, const mg_state S,
                                                         const mg_outputs O, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const double p1 = S.p1[i], v1 = S.v1[i], p2 = S.p2[i], v2 = S.v2[i];
  double x1, y1, x2, y2, o[kObs];
  lon2coord(P, p1, true, x1, y1);
  lon2coord(P, p2, false, x2, y2);
  observe(P, p1, v1, p2, v2, x1, y1, x2, y2, o);
  if (O.obs) {
#pragma unroll
    for (int k = 0; k < kObs; ++k) O.obs[i * kObs + k] = static_cast<float>(o[k]);
  }
  if (O.rec64) {
#pragma unroll
    for (int k = 0; k < kObs; ++k) O.rec64[i].obs[k] = o[k];
  }
  uint8_t* coll = O.flags ? O.flags + 4 * i + 3 : (O.coll ? O.coll + i : nullptr);
  if (coll) *coll = boxes_intersect(vehicle_box(P, y1, x1), vehicle_box(P, y2, x2)) ? 1 : 0;
}

// ============================================================================ replay memory
// The DQN replay memory (scripts/main.py:91-92 np.zeros((MEMORY_CAPACITY, 2*NUM_STATES+2)),
// :115-119 store_transition, :130-135 the minibatch draw). A batch of T x n transitions is
// appended in (t, i) order with three launches (kernel boundaries publish the partial sums;
// a last-arriver ticket with device-scope fences measured 8 % slower for the whole store):
//   replay_scan_kernel        one wave per 64 "write blocks" (t, 256-env slice): keep counts
//                             straight from the won bits, a wave scan (in-group offsets), the
//                             group's total;
//   replay_group_scan_kernel  one wave: group totals -> ring positions, memory_counter advanced;
//   replay_write_kernel       one block per 256 envs x kRTChunk steps, the step's
//                             observation kept in registers as the next transition's s; rows
//                             gathered in LDS in ring order and written as contiguous 8-byte
//                             stores (a row is 88 B: 16-byte alignment alternates).
// Rows are kRow floats [s(10), a, r, s'(10)], or kRowGoal [goal, s(10), a, r, next_goal, s'(10)]
// for hdqn.py's lower-level memory (:158, :180-184; goal_state = [goal] + state at :291, :304).
constexpr int kRow = 2 * kObs + 2;       // 22
constexpr int kRowGoal = 2 * kObs + 4;   // 24
constexpr int kRBlock = 256;        // envs per write block
constexpr int kRTChunk = 2;         // steps one write block walks (obs carried in registers; 1 step
                                    // measured +6 %, all 16 per block +11 %: DESIGN.md section 4)
constexpr int kRGroup = 64;         // write blocks per scan wave

struct ReplayIn {
  mg_transitions X;
  int64_t n;
  int64_t words;  // ceil(n / 64): won-mask words per step
  int64_t nbx;    // ceil(n / 256): write blocks per step
  int64_t nb;     // nbx * T
  int32_t T;
  int32_t skip_won;
};

struct ReplayScratch {  // carved from the caller's scratch buffer (8-byte header reserved)
  uint64_t* group_base;  // [ngroups] memory_counter before the group's first transition
  uint32_t* local;       // [nb] transitions of earlier write blocks of the same group
  uint32_t* group_total; // [ngroups]
};

__host__ __device__ inline int64_t replay_groups(int64_t nb) { return (nb + kRGroup - 1) / kRGroup; }

__host__ __device__ inline ReplayScratch replay_scratch(void* base, int64_t nb) {
  const int64_t ng = replay_groups(nb);
  ReplayScratch S;
  S.group_base = static_cast<uint64_t*>(base) + 1;
  S.local = reinterpret_cast<uint32_t*>(S.group_base + ng);
  S.group_total = S.local + nb;
  return S;
}

__device__ __forceinline__ bool replay_keep(const ReplayIn& R, int t, int64_t i) {
  if (i >= R.n) return false;
  if (!R.skip_won || R.X.won_mask == nullptr) return true;
  const uint64_t w = R.X.won_mask[static_cast<int64_t>(t) * R.words + (i >> 6)];
  return ((w >> (i & 63)) & 1u) == 0;
}

// Kept transitions of write block (t, bx).
__device__ __forceinline__ uint32_t replay_block_count(const ReplayIn& R, int t, int64_t bx) {
  const int64_t i0 = bx * kRBlock;
  const int64_t live = R.n - i0 < kRBlock ? R.n - i0 : kRBlock;
  if (!R.skip_won || R.X.won_mask == nullptr) return static_cast<uint32_t>(live);
  const uint64_t* w = R.X.won_mask + static_cast<int64_t>(t) * R.words + (i0 >> 6);
  uint64_t wk[kRBlock / 64];
#pragma unroll
  for (int k = 0; k < kRBlock / 64; ++k) wk[k] = live > 64 * k ? w[k] : ~0ull;  // loads issued together
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kRBlock / 64; ++k) {
    const int64_t v = live - 64 * k;  // live envs of this word
    const uint64_t m = v >= 64 ? ~0ull : (v <= 0 ? 0ull : ((1ull << v) - 1));
    c += __popcll(~wk[k] & m);
  }
  return c;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(v, off);
    if (lane >= off) v += u;
  }
  return v;
}

// One wave: group_base[g] = counter + sum(group_total[0..g)), then counter += sum.
__device__ __forceinline__ void replay_group_scan(const ReplayScratch& S, int64_t ng, uint64_t* counter) {
  const int lane = threadIdx.x & 63;
  const uint64_t c0 = *counter;
  uint64_t carry = 0;
  constexpr int kBatch = 16;  // loads issued together, then scanned: one memory wait per batch
  for (int64_t g0 = 0; g0 < ng; g0 += 64 * kBatch) {
    uint32_t v[kBatch];
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int64_t g = g0 + 64 * b + lane;
      v[b] = g < ng ? __atomic_load_n(S.group_total + g, __ATOMIC_RELAXED) : 0u;
    }
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int64_t g = g0 + 64 * b + lane;
      const uint32_t gi = wave_incl_scan(v[b]);
      if (g < ng) S.group_base[g] = c0 + carry + (gi - v[b]);
      carry += __shfl(gi, 63);
    }
  }
  if (lane == 0) *counter = c0 + carry;
}

__global__ __launch_bounds__(64) void replay_group_scan_kernel(const ReplayScratch S, int64_t ng,
                                                               uint64_t* counter) {
  replay_group_scan(S, ng, counter);
}

__global__ __launch_bounds__(64) void replay_scan_kernel(const ReplayIn R, ReplayScratch S) {
  const int lane = threadIdx.x;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * kRGroup + lane;
  uint32_t c = 0;
  if (b < R.nb) c = replay_block_count(R, static_cast<int>(b / R.nbx), b % R.nbx);
  const uint32_t incl = wave_incl_scan(c);
  if (b < R.nb) S.local[b] = incl - c;
  if (lane == 63) S.group_total[blockIdx.x] = incl;
}

// Rank of the calling thread among the block's kept threads, and the block total.
__device__ __forceinline__ int block_rank(bool keep, int* wave_cnt, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t m = __ballot(keep);
  const int below = __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
  if (lane == 0) wave_cnt[wave] = __popcll(m);
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < kRBlock / 64; ++w) {
    before += (w < wave) ? wave_cnt[w] : 0;
    total += wave_cnt[w];
  }
  return before + below;
}

__device__ __forceinline__ void load_row10(const float* src, float (&v)[kObs]) {
  const f32x2* s2 = reinterpret_cast<const f32x2*>(src);
#pragma unroll
  for (int k = 0; k < kObs / 2; ++k) {
    const f32x2 a = s2[k];
    v[2 * k] = a[0];
    v[2 * k + 1] = a[1];
  }
}

// KIND 0: main.py's DQN rows [s, a, r, s']; 1: hdqn.py's lower-level goal rows
// [goal, s, a, r, next_goal, s']; 2: Goal_DQN's rows [s', meta_goal, r, s'] (hdqn.py:97-101 at
// :325, where state is already next_state).
template <int KIND>
__global__ __launch_bounds__(kRBlock) void replay_write_kernel(const ReplayIn R, const ReplayScratch S,
                                                               const uint64_t* counter, float* rows,
                                                               int64_t cap) {
  constexpr bool GOAL = KIND == 1;
  constexpr bool META = KIND == 2;
  constexpr int kRow = GOAL ? kRowGoal : 2 * kObs + 2;  // floats per row
  constexpr int kS = GOAL ? 1 : 0;                      // column of s[0]
  constexpr int kS2 = kS + kObs + 2 + kS;               // column of s'[0]
  __shared__ __attribute__((aligned(16))) float tile[kRBlock * kRow];
  __shared__ int wave_cnt[kRBlock / 64];
  const int64_t bx = blockIdx.x;
  const int64_t i = bx * kRBlock + threadIdx.x;
  const bool live = i < R.n;
  const int t0 = blockIdx.y * kRTChunk;
  const int t1 = t0 + kRTChunk < R.T ? t0 + kRTChunk : R.T;
  const uint64_t end = *counter;  // memory_counter after this whole store
  // Only the newest `cap` transitions survive sequential stores; they occupy distinct slots,
  // so no two writes of this launch collide.
  const uint64_t first = end > static_cast<uint64_t>(cap) ? end - static_cast<uint64_t>(cap) : 0u;
  float s[kObs], o[kObs];
  if (live) {
    load_row10(t0 == 0 ? R.X.obs_first + i * kObs : R.X.obs + ((t0 - 1) * R.n + i) * kObs, s);
    load_row10(R.X.obs + (t0 * R.n + i) * kObs, o);
  }
  for (int t = t0; t < t1; ++t) {
    const int64_t row = static_cast<int64_t>(t) * R.n + i;
    const bool keep = replay_keep(R, t, i);
    float on[kObs];  // next step's row in flight while this step is gathered and written
    if (live && t + 1 < t1) load_row10(R.X.obs + (row + R.n) * kObs, on);
    int total;
    const int rank = block_rank(keep, wave_cnt, total);
    if (total > 0) {  // uniform across the block
      const int64_t b = static_cast<int64_t>(t) * R.nbx + bx;
      const uint64_t base = S.group_base[b / kRGroup] + S.local[b];
      if (keep) {
        float* d = tile + rank * kRow;
        const bool done = R.X.flags ? R.X.flags[4 * row + 2] != 0 : (R.X.done != nullptr && R.X.done[row] != 0);
        float s2[kObs];
        if (done && R.X.final_obs)
          load_row10(R.X.final_obs + row * kObs, s2);
        else
#pragma unroll
          for (int k = 0; k < kObs; ++k) s2[k] = o[k];
#pragma unroll
        for (int k = 0; k < kObs; ++k) {
          d[kS + k] = META ? s2[k] : s[k];
          d[kS2 + k] = s2[k];
        }
        if constexpr (META)
          d[kS + kObs] = R.X.meta_goal[row];
        else
          d[kS + kObs] = static_cast<float>(R.X.flags ? static_cast<int8_t>(R.X.flags[4 * row]) : R.X.a1[row]);
        d[kS + kObs + 1] = R.X.reward ? R.X.reward[row] : R.X.rew[2 * row];
        if constexpr (GOAL) {
          d[0] = R.X.goal[row];
          d[kS2 - 1] = R.X.next_goal[row];
        }
      }
      __syncthreads();
      const int skip = base >= first ? 0 : static_cast<int>(min<uint64_t>(first - base, total));
      const uint64_t slot0 = (base + skip) % static_cast<uint64_t>(cap);
      const int cnt = total - skip;  // <= cap: at most one wrap
      // the kept rows are one contiguous byte run of the ring (two at a wrap): an 8-byte head
      // when the run starts off 16-byte alignment, then 16-byte stores, then an 8-byte tail
      const int n_a = static_cast<int>(min<uint64_t>(static_cast<uint64_t>(cnt), static_cast<uint64_t>(cap) - slot0));
#pragma unroll
      for (int run = 0; run < 2; ++run) {
        const int r0 = run == 0 ? 0 : n_a, nr = run == 0 ? n_a : cnt - n_a;
        if (nr <= 0) continue;  // uniform
        float* d = rows + (run == 0 ? slot0 : 0) * kRow;
        const float* sp = tile + (skip + r0) * kRow;
        const int nf = nr * kRow;
        const int hd = (reinterpret_cast<uintptr_t>(d) & 15) ? 2 : 0;
        const int nb = (nf - hd) >> 2;
        const int tl = nf - hd - 4 * nb;  // 0 or 2
        if (threadIdx.x == 0 && hd) st_out(reinterpret_cast<f32x2*>(d), *reinterpret_cast<const f32x2*>(sp));
        if (threadIdx.x == 1 && tl)
          st_out(reinterpret_cast<f32x2*>(d + nf - 2), *reinterpret_cast<const f32x2*>(sp + nf - 2));
        const f32x2* s2 = reinterpret_cast<const f32x2*>(sp + hd);  // 8-byte aligned in LDS
        f32x4* d4 = reinterpret_cast<f32x4*>(d + hd);
        for (int k = threadIdx.x; k < nb; k += kRBlock) {
          const f32x2 lo = s2[2 * k], hi = s2[2 * k + 1];
          st_out(d4 + k, f32x4{lo[0], lo[1], hi[0], hi[1]});
        }
      }
    }
    __syncthreads();  // tile and wave counts are reused by the next step
#pragma unroll
    for (int k = 0; k < kObs; ++k) s[k] = o[k];
#pragma unroll
    for (int k = 0; k < kObs; ++k) o[k] = on[k];
  }
}

__global__ __launch_bounds__(kBlock) void replay_sample_kernel(const float* rows,
                                                               const uint64_t* counter, int64_t cap,
                                                               int row_floats, uint64_t seed, uint64_t draw,
                                                               int32_t filled_only, float* out,
                                                               int64_t* idx_out, int64_t batch) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (b >= batch) return;
  uint64_t m = static_cast<uint64_t>(cap);
  if (filled_only) {
    const uint64_t c = *counter;
    m = c < m ? c : m;
    if (m == 0) m = 1;
  }
  const uint4 u = philox4x32_10(
      make_uint4(static_cast<uint32_t>(b), static_cast<uint32_t>(static_cast<uint64_t>(b) >> 32),
                 static_cast<uint32_t>(draw), static_cast<uint32_t>(draw >> 32)),
      static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
  const uint64_t idx = (static_cast<uint64_t>(u.x) * m) >> 32;
  if (idx_out) idx_out[b] = static_cast<int64_t>(idx);
  const f32x2* src = reinterpret_cast<const f32x2*>(rows + idx * row_floats);
  f32x2* dst = reinterpret_cast<f32x2*>(out + b * row_floats);
  for (int k = 0; k < row_floats / 2; ++k) dst[k] = src[k];
}

thread_local char g_err[512] = "";
// mg_time_next_launch: events the next step launch of this thread records at its dispatch
thread_local hipEvent_t g_ev_start = nullptr;
thread_local hipEvent_t g_ev_stop = nullptr;

int fail(int code, const char* fmt, const char* what) {
  std::snprintf(g_err, sizeof(g_err), fmt, what);
  return code ? code : static_cast<int>(hipErrorInvalidValue);
}

int check_state(const mg_state* s) {
  if (!s || !s->p1 || !s->v1 || !s->p2 || !s->v2 || !s->ret1 || !s->ret2 || !s->tf)
    return fail(hipErrorInvalidValue, "%s", "mg_state has a NULL array");
  return 0;
}

int check_common(const mg_params* p, const mg_state* s, const mg_outputs* o, int64_t n) {
  if (!p) return fail(hipErrorInvalidValue, "%s", "params is NULL");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (n > (static_cast<int64_t>(0x7fffffff) * kBlock))
    return fail(hipErrorInvalidValue, "%s", "n exceeds the grid limit");
  if (int e = check_state(s)) return e;
  if (!o) return fail(hipErrorInvalidValue, "%s", "outputs is NULL (pass a zeroed mg_outputs)");
  if (o->obs && (reinterpret_cast<uintptr_t>(o->obs) & 15))
    return fail(hipErrorInvalidValue, "%s", "obs must be 16-byte aligned");
  if (o->rew && (reinterpret_cast<uintptr_t>(o->rew) & 7))
    return fail(hipErrorInvalidValue, "%s", "rew must be 8-byte aligned");
  if (o->flags) {
    if (reinterpret_cast<uintptr_t>(o->flags) & 3)
      return fail(hipErrorInvalidValue, "%s", "flags must be 4-byte aligned");
    if (o->done || o->coll || o->rec64)
      return fail(hipErrorInvalidValue, "%s", "flags replaces done / coll (and rec64 has its own status): pass NULL");
  }
  return 0;
}

int finish_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  g_err[0] = '\0';
  return 0;
}

template <int ACT>
int launch_step(const Launch& L, hipStream_t stream, const char* what) {
  const unsigned blocks = static_cast<unsigned>((L.n + kBlock - 1) / kBlock);
  hipEvent_t start = g_ev_start, stop = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  if (start || stop) {  // profiling: the dispatch packet itself records both events
    if (L.O.rec64)
      hipExtLaunchKernelGGL((step_kernel<ACT, true>), dim3(blocks), dim3(kBlock), 0, stream, start,
                            stop, 0, L);
    else
      hipExtLaunchKernelGGL((step_kernel<ACT, false>), dim3(blocks), dim3(kBlock), 0, stream, start,
                            stop, 0, L);
  } else if (L.O.rec64) {
    hipLaunchKernelGGL((step_kernel<ACT, true>), dim3(blocks), dim3(kBlock), 0, stream, L);
  } else {
    hipLaunchKernelGGL((step_kernel<ACT, false>), dim3(blocks), dim3(kBlock), 0, stream, L);
  }
  return finish_launch(what);
}

int launch_rollout(const Rollout& R, hipStream_t stream) {
  const unsigned blocks = static_cast<unsigned>((R.n + kBlock - 1) / kBlock);
  hipEvent_t start = g_ev_start, stop = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  const bool full = R.T.obs && R.T.rew && R.T.flags && R.St.rec &&
                    (R.flags & MG_AUTORESET);
  if (start || stop) {
    if (full)
      hipExtLaunchKernelGGL(rollout_kernel<true>, dim3(blocks), dim3(kBlock), 0, stream, start, stop, 0, R);
    else
      hipExtLaunchKernelGGL(rollout_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, start, stop, 0, R);
  } else if (full) {
    hipLaunchKernelGGL(rollout_kernel<true>, dim3(blocks), dim3(kBlock), 0, stream, R);
  } else {
    hipLaunchKernelGGL(rollout_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, R);
  }
  return finish_launch("mg_rollout_random");
}

// The constants of mpc_1d's equality step (helper.py:152-191) in the operation order of quadprog
// 0.1.11's qpgen2 (Goldfarb-Idnani; helper.py:182 -> qpsolvers 1.8.0 -> quadprog.solve_qp with
// G = P, C = -A[1]', b = -B, meq = 1), file compiled without contraction:
//   n = A[1] = (dt, ..., dt), dt = t / 10 (the velocity row of [a^9 b, ..., b]);
//   P = D'D + 0.01 I, D the 9 x 10 first-difference operator (integer sums, then + 0.01);
//   dpofa: P = R'R, column by column, s accumulating t*t before a(j,j) - s;
//   dpori: J = R^-1 in place (a(k,k) = 1 / a(k,k), column k scaled by -a(k,k), then
//          a(1:k, j) += a(k, j) a(1:k, k) for j > k);
//   d = J'n (d_i = sum_j J(j,i) n_j), z = J d (z_i = sum_j J(i,j) d_j, accumulated in j order),
//   z'n (sum in index order).
// The residual's sign only negates n, d, z and the step exactly, so u0 = (b / z'n) z0 for either
// sign of b = vt - v0. Restated from the published algorithm (LINPACK dpofa / dpori and
// Goldfarb & Idnani 1983 as coded in Turlach's solve.QP.f); quadprog is not in this image.
void mpc_qp_constants(double t, double* nz_out, double* z0_out, double* vsmall_out) {
  constexpr int kT = 10;
  const double dt = t / kT;
  double n[kT], a[kT][kT] = {}, d[kT], z[kT];  // a[i][j] = LINPACK's a(i+1, j+1)
  for (int i = 0; i < kT; ++i) n[i] = 0.0 * 0.0 + 1.0 * dt;  // row [0 1] of a^k times b
  for (int i = 0; i + 1 < kT; ++i) {
    a[i][i] += 1.0;
    a[i + 1][i + 1] += 1.0;
    a[i][i + 1] -= 1.0;
    a[i + 1][i] -= 1.0;
  }
  for (int i = 0; i < kT; ++i) a[i][i] += 0.01;
  for (int j = 0; j < kT; ++j) {  // dpofa (upper triangle)
    double s = 0.0;
    for (int k = 0; k < j; ++k) {
      double dot = 0.0;
      for (int l = 0; l < k; ++l) dot = dot + a[l][k] * a[l][j];
      double tk = a[k][j] - dot;
      tk = tk / a[k][k];
      a[k][j] = tk;
      s = s + tk * tk;
    }
    s = a[j][j] - s;
    a[j][j] = std::sqrt(s);
  }
  for (int k = 0; k < kT; ++k) {  // dpori
    a[k][k] = 1.0 / a[k][k];
    const double tk = -a[k][k];
    for (int i = 0; i < k; ++i) a[i][k] = tk * a[i][k];
    for (int j = k + 1; j < kT; ++j) {
      const double tj = a[k][j];
      a[k][j] = 0.0;
      if (tj == 0.0) continue;  // daxpy returns early for a zero multiplier
      for (int i = 0; i <= k; ++i) a[i][j] = a[i][j] + tj * a[i][k];
    }
  }
  for (int i = 0; i < kT; ++i) {  // d = J'n (J is upper triangular: a[j][i] = 0 for j > i)
    double s = 0.0;
    for (int j = 0; j < kT; ++j) s = s + (j <= i ? a[j][i] : 0.0) * n[j];
    d[i] = s;
  }
  for (int i = 0; i < kT; ++i) z[i] = 0.0;
  for (int j = 0; j < kT; ++j)  // z = J d
    for (int i = 0; i < kT; ++i) z[i] = z[i] + (i <= j ? a[i][j] : 0.0) * d[j];
  double nz = 0.0;
  for (int i = 0; i < kT; ++i) nz = nz + z[i] * n[i];
  // qpgen2's machine-precision probe: a constraint residual below vsmall is set to 0
  volatile double vs = 1e-60;
  for (;;) {
    vs = vs + vs;
    const double ta = vs * 0.1 + 1.0, tb = vs * 0.2 + 1.0;
    if (ta > 1.0 && tb > 1.0) break;
  }
  *nz_out = nz;
  *z0_out = z[0];
  *vsmall_out = vs;
}

// ============================================================================ statistics reduction
// The per-env 64-byte records (mg_episode_stats) summed to one mg_stats_totals in a FIXED order, so
// the fp64 sums are reproducible bit for bit (oracle/merge_oracle.py stats_reduce_fixed restates it):
//   pass 1 (block b of kRedThreads threads, kRedEnvs envs): thread t adds the records of envs
//          b kRedEnvs + j kRedThreads + t, j = 0..kRedPer-1, in j order onto -0.0 (the additive
//          identity), then the block folds its kRedThreads values in halves (v[t] += v[t + o],
//          o = 128, 64, ..., 1) -> partial b;
//   pass 2 (one block): thread t adds partials t, t + 256, ... in order onto -0.0, then the same fold.
// The counts are exact int64 sums; the fp64 ones are ret[0], ret[1], ret_main and q_eval. Replaces the logging loops' running totals (hdqn.py:330-346,
// main.py:221-228) for a whole batch; a torch sum over strided record columns took 7.6 ms at 2^20
// envs (BENCH_r03 episodes.reduce_ms) for 64 MB of records.
constexpr int kRedThreads = 256;
constexpr int kRedPer = 4;
constexpr int kRedEnvs = kRedThreads * kRedPer;  // 1,024 records (64 KB) per pass-1 block

constexpr int kRedSums = 4;  // ret[0], ret[1], ret_main, q_eval

__device__ __forceinline__ void red_fold(double (*sd)[kRedThreads], int64_t (*si)[kRedThreads], int t) {
#pragma unroll
  for (int o = kRedThreads / 2; o > 0; o >>= 1) {
    __syncthreads();
    if (t < o) {
#pragma unroll
      for (int k = 0; k < kRedSums; ++k) sd[k][t] = sd[k][t] + sd[k][t + o];
#pragma unroll
      for (int k = 0; k < 6; ++k) si[k][t] += si[k][t + o];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void red_store(mg_stats_totals* out, double (*sd)[kRedThreads],
                                          int64_t (*si)[kRedThreads]) {
  mg_stats_totals o;
#pragma unroll
  for (int k = 0; k < 3; ++k) o.ret[k] = sd[k][0];
  o.q_eval = sd[3][0];
#pragma unroll
  for (int k = 0; k < 6; ++k) o.counts[k] = si[k][0];
  *out = o;
}

__global__ __launch_bounds__(kRedThreads) void stats_reduce_kernel(const mg_episode_stats* rec, int64_t n,
                                                                   mg_stats_totals* part) {
  __shared__ double sd[kRedSums][kRedThreads];
  __shared__ int64_t si[6][kRedThreads];
  const int t = threadIdx.x;
  double a0 = -0.0, a1 = -0.0, a2 = -0.0, a3 = -0.0;
  int64_t c[6] = {0, 0, 0, 0, 0, 0};
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRedEnvs + t;
#pragma unroll
  for (int j = 0; j < kRedPer; ++j) {
    const int64_t i = base + j * kRedThreads;
    if (i < n) {
      // the record as four 16-byte loads: {ret[0], ret[1]}, {ret_main, pending}, counts 0-3, 4-7
      const f64x2* r2 = reinterpret_cast<const f64x2*>(rec + i);
      const f64x2 f0 = __builtin_nontemporal_load(r2), f1 = __builtin_nontemporal_load(r2 + 1);
      const u32x4* u = reinterpret_cast<const u32x4*>(rec + i) + 2;
      const u32x4 u0 = __builtin_nontemporal_load(u), u1 = __builtin_nontemporal_load(u + 1);
      a0 = a0 + f0.x;
      a1 = a1 + f0.y;
      a2 = a2 + f1.x;
      a3 = a3 + __builtin_bit_cast(double, (static_cast<uint64_t>(u1.w) << 32) | u1.z);
      c[0] += u0.x;
      c[1] += u0.y;
      c[2] += u0.z;
      c[3] += u0.w;
      c[4] += u1.x;
      c[5] += u1.y;
    }
  }
  sd[0][t] = a0;
  sd[1][t] = a1;
  sd[2][t] = a2;
  sd[3][t] = a3;
#pragma unroll
  for (int k = 0; k < 6; ++k) si[k][t] = c[k];
  red_fold(sd, si, t);
  if (t == 0) red_store(part + blockIdx.x, sd, si);
}

__global__ __launch_bounds__(kRedThreads) void stats_reduce_final_kernel(const mg_stats_totals* part, int64_t nb,
                                                                         mg_stats_totals* out) {
  __shared__ double sd[kRedSums][kRedThreads];
  __shared__ int64_t si[6][kRedThreads];
  const int t = threadIdx.x;
  double a[kRedSums] = {-0.0, -0.0, -0.0, -0.0};
  int64_t c[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t k = t; k < nb; k += kRedThreads) {
    const mg_stats_totals p = part[k];
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = a[q] + p.ret[q];
    a[3] = a[3] + p.q_eval;
#pragma unroll
    for (int q = 0; q < 6; ++q) c[q] += p.counts[q];
  }
#pragma unroll
  for (int q = 0; q < kRedSums; ++q) sd[q][t] = a[q];
#pragma unroll
  for (int q = 0; q < 6; ++q) si[q][t] = c[q];
  red_fold(sd, si, t);
  if (t == 0) red_store(out, sd, si);
}

// goal_status of n (dx1, v2) pairs, the function the h-DQN kernel evaluates (tests, evaluation)
__global__ __launch_bounds__(kBlock) void goal_status_kernel(const double* dx1, const double* v2, int8_t* out,
                                                             int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = static_cast<int8_t>(goal_status(dx1[i], v2[i]));
}

// ============================================================================ host (CPU) path
// The step kernel's per-env body on the host, over host pointers: the single env of BASELINE
// config 1 (MergeEnv.step / reset / observe, merging_env.py:118-230, driven one step at a time by
// scripts/human_player.py:112-187 at 20 Hz), where a kernel launch plus a stream synchronisation
// per step (28.5 us, BENCH_r03 dropin_single_env) costs 20x the step's own ~1 us of fp64 work.
// The same MG_HD functions as the kernels, so a host step gives the kernel's doubles bit for bit
// (tests/test_dropin.py: golden traces on the CPU; test_host_step_equals_kernel on the GPU box).
// Outputs and their conditions follow step_kernel<kActArrays, OUT64 = rec64 != NULL> exactly.
void host_step_env(const Launch& L, int64_t i, bool& done, bool& won) {
  const mg_params& P = L.P;
  const int a1 = L.a1[i];
  const int a2 = L.a2 ? static_cast<int>(L.a2[i]) : MG_ACTION_NONE;
  Env e = load_env(L.S, i);
  StepOut r;
  env_step_sp(P, e, a1, a2, action_speed_or0(P, a1), action_speed_or0(P, a2), r);
  done = won = false;
  if (r.bad) {
    if (L.O.error) *L.O.error |= r.bad;
    store_env(L.S, i, e);
  } else {
    if (L.O.rec64) {
      mg_rec64* rec = L.O.rec64 + i;
      double x1, y1, x2, y2, od[kObs];
      lon2coord(P, e.p1, true, x1, y1);
      lon2coord(P, e.p2, false, x2, y2);
      observe(P, e.p1, e.v1, e.p2, e.v2, x1, y1, x2, y2, od);
      for (int k = 0; k < kObs; ++k) rec->obs[k] = od[k];
      rec->rew[0] = r.r1;
      rec->rew[1] = r.r2;
      rec->acc[0] = r.acc1;
      rec->acc[1] = r.acc2;
      rec->pos[0] = e.p1;
      rec->pos[1] = e.p2;
      rec->vel[0] = e.v1;
      rec->vel[1] = e.v2;
      rec->ret[0] = e.ret1;
      rec->ret[1] = e.ret2;
      rec->tf = pack_tf(e);
      rec->status = (r.done ? MG_ST_DONE : 0u) | (r.coll ? MG_ST_COLLISION : 0u) |
                    (r.r1_int ? MG_ST_R1_INT : 0u) | (r.r2_int ? MG_ST_R2_INT : 0u) |
                    (r.v1_int ? MG_ST_V1_INT : 0u) | (r.v2_int ? MG_ST_V2_INT : 0u);
    } else if (L.O.rew) {
      L.O.rew[2 * i] = static_cast<float>(r.r1);
      L.O.rew[2 * i + 1] = static_cast<float>(r.r2);
    }
    if (L.O.flags) {
      reinterpret_cast<uint32_t*>(L.O.flags)[i] = pack_step_bytes(a1, a2, r.done, r.coll);
    } else {
      if (L.O.done) L.O.done[i] = r.done ? 1 : 0;
      if (L.O.coll) L.O.coll[i] = r.coll ? 1 : 0;
    }
    done = r.done;
    won = e.winner == 1;
    after_step(P, e, r, L.St, L.O.final_obs ? L.O.final_obs + i * kObs : nullptr, i,
               (L.flags & MG_AUTORESET) != 0, nullptr, &L.R0);
    store_env(L.S, i, e);
  }
  if (!L.O.rec64 && L.O.obs) {  // the kernel's observation tile: zeros for a bad action's env
    for (int k = 0; k < kObs; ++k) L.O.obs[i * kObs + k] = r.o[k];
  }
}

void host_reset_env(const mg_params& P, const mg_state& S, const mg_outputs& O, int64_t i) {
  S.p1[i] = S.p2[i] = P.start_point;
  S.v1[i] = S.v2[i] = P.start_vel;
  S.ret1[i] = S.ret2[i] = 0.0;
  S.tf[i] = 0u;
  if (!O.obs && !O.rec64) return;
  double o[kObs];
  reset_obs(P, o);
  if (O.obs)
    for (int k = 0; k < kObs; ++k) O.obs[i * kObs + k] = static_cast<float>(o[k]);
  if (O.rec64) {
    mg_rec64* rec = O.rec64 + i;
    std::memset(rec, 0, sizeof(*rec));
    for (int k = 0; k < kObs; ++k) rec->obs[k] = o[k];
    rec->pos[0] = rec->pos[1] = P.start_point;
    rec->vel[0] = rec->vel[1] = P.start_vel;
  }
}

void host_observe_env(const mg_params& P, const mg_state& S, const mg_outputs& O, int64_t i) {
  const double p1 = S.p1[i], v1 = S.v1[i], p2 = S.p2[i], v2 = S.v2[i];
  double x1, y1, x2, y2, o[kObs];
  lon2coord(P, p1, true, x1, y1);
  lon2coord(P, p2, false, x2, y2);
  observe(P, p1, v1, p2, v2, x1, y1, x2, y2, o);
  if (O.obs)
    for (int k = 0; k < kObs; ++k) O.obs[i * kObs + k] = static_cast<float>(o[k]);
  if (O.rec64)
    for (int k = 0; k < kObs; ++k) O.rec64[i].obs[k] = o[k];
  uint8_t* coll = O.flags ? O.flags + 4 * i + 3 : (O.coll ? O.coll + i : nullptr);
  if (coll) *coll = boxes_intersect(vehicle_box(P, y1, x1), vehicle_box(P, y2, x2)) ? 1 : 0;
}

}  // namespace

// one config-5 launch (with dispatch-packet events when mg_time_next_launch armed them)
template <int OPP, bool CHECKED>
static void launch_qnet(int64_t blocks, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, const QRollout& R) {
  if (ev0 || ev1)
    hipExtLaunchKernelGGL((qnet_rollout_ws_kernel<OPP, CHECKED>), dim3(blocks), dim3(kQWsThreads), 0, st, ev0, ev1, 0, R);
  else
    hipLaunchKernelGGL((qnet_rollout_ws_kernel<OPP, CHECKED>), dim3(blocks), dim3(kQWsThreads), 0, st, R);
}

extern "C" {

int mg_abi_version(void) { return MG_ABI_VERSION; }


int mg_time_next_launch(void* start_event, void* stop_event) {
  g_ev_start = static_cast<hipEvent_t>(start_event);
  g_ev_stop = static_cast<hipEvent_t>(stop_event);
  return 0;
}

const char* mg_last_error(void) { return g_err; }

// The compiler that built this library (its hipcc version decides the inline-asm permlane hazard
// padding of qnet_gather_q, which hipcc 7.2's builtins miscompiled): printed in the GPU test log
// header and the bench line.
#ifndef MG_SRC_SHA
#define MG_SRC_SHA "unknown"  // merging_gym/build.py passes the sha256 of source + header + flags
#endif
const char* mg_build_info(void) {
  return "clang " __clang_version__ "; HIP " MG_STR(HIP_VERSION_MAJOR) "." MG_STR(HIP_VERSION_MINOR) "."
         MG_STR(HIP_VERSION_PATCH) "; ABI " MG_STR(MG_ABI_VERSION) "; gfx950, -ffp-contract=off; src " MG_SRC_SHA;
}

void mg_params_default(mg_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->R = 30000.0;
  p->H = 1000.0;
  p->W = 300.0;
  p->dT = 0.2;
  p->r_first = 2.0;
  p->r_second = 1.0;
  p->r_collision = -10.0;
  p->vel_penalty = 0.001;
  p->time_penalty = 0.0;
  p->start_point = 50.0;
  p->end_point = 950.0;
  p->start_vel = 20.0;
  p->vel_ref = 20.0;
  p->prediction_t = 3.0;
  volatile double h = 1000.0, r = 30000.0;  // libm at run time, as np.arctan2 does
  p->angle0 = std::atan2(h, r);                 // merging_env.py:49
  for (int k = 0; k < MG_NUM_ACTIONS; ++k) p->action_speed[k] = 10.0 * k;
  p->veh_w = 4;
  p->veh_h = 8;
  p->timeout_steps = 2501;
  p->inv_R = 1.0 / p->R;
  mpc_qp_constants(p->prediction_t, &p->qp_nz, &p->qp_z0, &p->qp_vsmall);
  p->qp_inv_nz = 1.0 / p->qp_nz;
}

int mg_goal_status(const double* dx1, const double* v2, int8_t* status, int64_t n, void* stream) {
  if (!dx1 || !v2 || !status) return fail(hipErrorInvalidValue, "%s", "mg_goal_status: NULL pointer");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (n == 0) return 0;
  hipLaunchKernelGGL(goal_status_kernel, dim3(static_cast<unsigned>((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), dx1, v2, status, n);
  return finish_launch("mg_goal_status");
}

int mg_step(const mg_params* params, const mg_state* state, const int8_t* a1, const int8_t* a2,
            const mg_outputs* out, const mg_stats* stats, int64_t n, uint32_t flags,
            void* stream) {
  if (int e = check_common(params, state, out, n)) return e;
  if (n == 0) return 0;
  if (!a1) return fail(hipErrorInvalidValue, "%s", "a1 is NULL");
  Launch L{};
  L.P = *params;
  L.R0 = reset0(*params);
  L.S = *state;
  L.O = *out;
  if (stats) L.St = *stats;
  L.a1 = a1;
  L.a2 = a2;
  L.n = n;
  L.flags = flags;
  return launch_step<kActArrays>(L, static_cast<hipStream_t>(stream), "mg_step");
}

int mg_step_random(const mg_params* params, const mg_state* state, int8_t* a1_out,
                   int8_t* a2_out, const mg_outputs* out, const mg_stats* stats, int64_t n,
                   int64_t env_offset, uint64_t seed, uint64_t step_idx, int32_t opponent_random, uint32_t flags,
                   void* stream) {
  if (int e = check_common(params, state, out, n)) return e;
  if (n == 0) return 0;
  Launch L{};
  L.P = *params;
  L.R0 = reset0(*params);
  L.S = *state;
  L.O = *out;
  if (stats) L.St = *stats;
  if (out->flags && (a1_out || a2_out))
    return fail(hipErrorInvalidValue, "%s", "flags records the actions: pass NULL a1_out / a2_out");
  L.a1_out = a1_out;
  L.a2_out = a2_out;
  L.seed = seed;
  L.step_idx = step_idx;
  L.env_offset = env_offset;
  L.opp_random = opponent_random;
  L.n = n;
  L.flags = flags;
  return launch_step<kActPhilox>(L, static_cast<hipStream_t>(stream), "mg_step_random");
}

int mg_rollout_random(const mg_params* params, const mg_state* state, const mg_traj* traj,
                      const mg_stats* stats, int64_t n, int64_t env_offset, uint64_t seed,
                      uint64_t first_step, int32_t num_steps, int32_t opponent_random,
                      uint32_t flags, void* stream) {
  mg_outputs none{};
  if (int e = check_common(params, state, &none, n)) return e;
  if (!traj) return fail(hipErrorInvalidValue, "%s", "traj is NULL (pass a zeroed mg_traj)");
  if (num_steps < 0 || num_steps > 65535)
    return fail(hipErrorInvalidValue, "%s", "need 0 <= num_steps <= 65535 (split longer rollouts)");
  if ((traj->obs && (reinterpret_cast<uintptr_t>(traj->obs) & 15)) ||
      (traj->final_obs && (reinterpret_cast<uintptr_t>(traj->final_obs) & 7)) ||
      (traj->rew && (reinterpret_cast<uintptr_t>(traj->rew) & 7)) ||
      (reinterpret_cast<uintptr_t>(traj->flags) & 3))
    return fail(hipErrorInvalidValue, "%s", "traj.obs must be 16-byte, rew/final_obs 8-byte, flags 4-byte aligned");
  if (n == 0 || num_steps == 0) return 0;
  Rollout R{};
  R.P = *params;
  R.R0 = reset0(*params);
  R.S = *state;
  R.T = *traj;
  if (stats) R.St = *stats;
  R.seed = seed;
  R.first_step = first_step;
  R.env_offset = env_offset;
  R.n = n;
  R.num_steps = num_steps;
  R.opp_random = opponent_random;
  R.flags = flags;
  return launch_rollout(R, static_cast<hipStream_t>(stream));
}

size_t mg_qnet_packed_bytes(void) { return static_cast<size_t>(kQNetBytes + kQ32NetBytes); }

int mg_qnet_pack(const float* fc1_w, const float* fc1_b, const float* fc2_w, const float* fc2_b,
                 const float* out_w, const float* out_b, int32_t in_dim, int32_t out_dim,
                 void* packed, void* stream) {
  if (!fc1_w || !fc1_b || !fc2_w || !fc2_b || !out_w || !out_b || !packed)
    return fail(hipErrorInvalidValue, "%s", "mg_qnet_pack: NULL pointer");
  if (in_dim < 1 || in_dim > kQMaxIn || out_dim < 1 || out_dim > 8)
    return fail(hipErrorInvalidValue, "%s", "mg_qnet_pack: need 1 <= in_dim <= 13, 1 <= out_dim <= 8");
  if (reinterpret_cast<uintptr_t>(packed) & 15)
    return fail(hipErrorInvalidValue, "%s", "mg_qnet_pack: packed buffer must be 16-byte aligned");
  const int total = kQFrags * 64 * 8;  // one thread per (fragment, lane, element)
  hipLaunchKernelGGL(qnet_pack_kernel, dim3((total + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), fc1_w, fc1_b, fc2_w, fc2_b, out_w, out_b,
                     in_dim, out_dim, static_cast<uint8_t*>(packed));
  // the 32x32 layout behind it (qnet32_mlp: the config-5 kernel without a net opponent)
  const int total32 = kQ32R1 * kQ32S1 + kQ32R2 * kQ32S2 + kQ32R3 * kQ32S3;
  hipLaunchKernelGGL(qnet32_pack_kernel, dim3((total32 + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), fc1_w, fc1_b, fc2_w, fc2_b, out_w, out_b,
                     in_dim, out_dim, static_cast<uint8_t*>(packed) + kQNetBytes);
  return finish_launch("mg_qnet_pack");
}

size_t mg_qnet_fragment_bytes(void) { return static_cast<size_t>(kQNetBytes); }

int mg_qnet_fragments(const void* packed, void* fragments, void* stream) {
  if (!packed || !fragments) return fail(hipErrorInvalidValue, "%s", "mg_qnet_fragments: NULL pointer");
  if ((reinterpret_cast<uintptr_t>(packed) | reinterpret_cast<uintptr_t>(fragments)) & 15)
    return fail(hipErrorInvalidValue, "%s", "mg_qnet_fragments: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(qnet_fragments_kernel, dim3(kQNetBytes / 1024), dim3(64), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(packed), static_cast<uint8_t*>(fragments));
  return finish_launch("mg_qnet_fragments");
}

int mg_qnet_forward(const void* packed, const float* x, int32_t in_dim, int32_t swap_halves, float* q,
                    int64_t n, void* stream) {
  if (!packed || !x || !q) return fail(hipErrorInvalidValue, "%s", "mg_qnet_forward: NULL pointer");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (in_dim < 1 || in_dim > kQMaxIn || (swap_halves && in_dim != kObs))
    return fail(hipErrorInvalidValue, "%s", "mg_qnet_forward: need 1 <= in_dim <= 13 (swap_halves: in_dim 10)");
  if (reinterpret_cast<uintptr_t>(packed) & 15)
    return fail(hipErrorInvalidValue, "%s", "packed net must be 16-byte aligned");
  if (n == 0) return 0;
  const unsigned blocks = static_cast<unsigned>((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(qnet_forward_kernel, dim3(blocks), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(packed), x, in_dim,
                     swap_halves, q, n);
  return finish_launch("mg_qnet_forward");
}

int mg_rollout_qnet(const mg_params* params, const mg_state* state, const mg_traj* traj,
                    const mg_stats* stats, int64_t n, int64_t env_offset, uint64_t seed,
                    uint64_t first_step, int32_t num_steps, const void* net, int32_t out_dim,
                    uint64_t greedy_threshold, int32_t opponent_mode,
                    uint64_t opp_greedy_threshold, const void* opp_net, uint32_t flags, void* stream) {
  mg_outputs none{};
  if (int e = check_common(params, state, &none, n)) return e;
  if (!traj) return fail(hipErrorInvalidValue, "%s", "traj is NULL (pass a zeroed mg_traj)");
  if (!net || (reinterpret_cast<uintptr_t>(net) & 15))
    return fail(hipErrorInvalidValue, "%s", "net must be a 16-byte aligned packed Q-net");
  if (num_steps < 0 || out_dim < 1 || out_dim > 8)
    return fail(hipErrorInvalidValue, "%s", "need num_steps >= 0 and 1 <= out_dim <= 8");
  if (opponent_mode < 0 || opponent_mode > 3)
    return fail(hipErrorInvalidValue, "%s",
                "opponent_mode must be 0 (None), 1 (uniform), 2 (same net) or 3 (opp_net)");
  if (opponent_mode == 3 && (!opp_net || (reinterpret_cast<uintptr_t>(opp_net) & 15)))
    return fail(hipErrorInvalidValue, "%s", "opponent_mode 3 needs opp_net, a 16-byte aligned packed Q-net");
  if ((traj->obs && (reinterpret_cast<uintptr_t>(traj->obs) & 15)) ||
      (traj->final_obs && (reinterpret_cast<uintptr_t>(traj->final_obs) & 7)) ||
      (traj->rew && (reinterpret_cast<uintptr_t>(traj->rew) & 7)) ||
      (reinterpret_cast<uintptr_t>(traj->flags) & 3))
    return fail(hipErrorInvalidValue, "%s", "traj.obs must be 16-byte, rew/final_obs 8-byte, flags 4-byte aligned");
  if (n == 0 || num_steps == 0) return 0;
  QRollout R{};
  R.P = *params;
  R.R0 = reset0(*params);
  R.S = *state;
  R.T = *traj;
  if (stats) R.St = *stats;
  R.net = static_cast<const uint8_t*>(net);
  R.opp_net = static_cast<const uint8_t*>(opp_net);
  R.seed = seed;
  R.first_step = first_step;
  R.greedy_thr = greedy_threshold;
  R.opp_greedy_thr = opp_greedy_threshold;
  R.env_offset = env_offset;
  R.n = n;
  R.num_steps = num_steps;
  R.out_dim = out_dim;
  R.flags = flags;
  R.fin = finish_bound(*params);
  const int64_t block_envs = opponent_mode == 3 ? qws_envs<3>() : qws_envs<0>();
  const unsigned blocks = static_cast<unsigned>((n + block_envs - 1) / block_envs);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipEvent_t ev0 = g_ev_start, ev1 = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  const bool checked = out_dim > MG_NUM_ACTIONS;  // argmax may name an action past action_dict
  if (opponent_mode == 0)
    checked ? launch_qnet<0, true>(blocks, st, ev0, ev1, R) : launch_qnet<0, false>(blocks, st, ev0, ev1, R);
  else if (opponent_mode == 1)
    checked ? launch_qnet<1, true>(blocks, st, ev0, ev1, R) : launch_qnet<1, false>(blocks, st, ev0, ev1, R);
  else if (opponent_mode == 2)
    launch_qnet<2, true>(blocks, st, ev0, ev1, R);
  else
    launch_qnet<3, true>(blocks, st, ev0, ev1, R);
  return finish_launch("mg_rollout_qnet");
}

int mg_rollout_hdqn(const mg_params* params, const mg_state* state, const mg_traj* traj,
                    const mg_hdqn_traj* htraj, const mg_stats* stats, int8_t* goal, int8_t* goal_op,
                    double* ext_acc, int64_t n, int64_t env_offset, uint64_t seed, uint64_t first_step,
                    int32_t num_steps,
                    const void* meta_net, int32_t num_goals, const void* lower_net, int32_t reset_goal,
                    uint64_t greedy_threshold, int32_t opponent_mode, const void* opp_meta_net,
                    const void* opp_lower_net, float* ring_rows,
                    uint64_t* ring_counter, int64_t ring_capacity, uint32_t flags, void* stream) {
  if (ring_rows && (!ring_counter || ring_capacity < 1 || (reinterpret_cast<uintptr_t>(ring_rows) & 15)))
    return fail(hipErrorInvalidValue, "%s", "ring_rows needs ring_counter, capacity >= 1 and 16-byte alignment");
  mg_outputs none{};
  if (int e = check_common(params, state, &none, n)) return e;
  if (!traj) return fail(hipErrorInvalidValue, "%s", "traj is NULL (pass a zeroed mg_traj)");
  if (!goal) return fail(hipErrorInvalidValue, "%s", "goal is NULL (an [n] int8 device array)");
  if (!meta_net || !lower_net || ((reinterpret_cast<uintptr_t>(meta_net) | reinterpret_cast<uintptr_t>(lower_net)) & 15))
    return fail(hipErrorInvalidValue, "%s", "meta_net / lower_net must be 16-byte aligned packed Q-nets");
  if (num_steps < 0 || num_goals < 1 || num_goals > 8 || reset_goal < 0 || reset_goal >= num_goals)
    return fail(hipErrorInvalidValue, "%s", "need num_steps >= 0, 1 <= num_goals <= 8, 0 <= reset_goal < num_goals");
  if (opponent_mode < 0 || opponent_mode > 3)
    return fail(hipErrorInvalidValue, "%s",
                "opponent_mode must be 0 (None), 1 (uniform), 2 (self-play) or 3 (other h-DQN)");
  if (opponent_mode >= 2 && !goal_op)
    return fail(hipErrorInvalidValue, "%s", "opponent_mode 2 / 3 needs goal_op (an [n] int8 device array)");
  if (opponent_mode == 3 &&
      (!opp_meta_net || !opp_lower_net ||
       ((reinterpret_cast<uintptr_t>(opp_meta_net) | reinterpret_cast<uintptr_t>(opp_lower_net)) & 15)))
    return fail(hipErrorInvalidValue, "%s",
                "opponent_mode 3 needs 16-byte aligned opp_meta_net / opp_lower_net (mg_qnet_fragments copies)");
  if (htraj && (htraj->ext_reward || htraj->no_break) && !ext_acc)
    return fail(hipErrorInvalidValue, "%s", "ext_reward / no_break need ext_acc (an [n] double device array)");
  if (htraj && htraj->no_break && (reinterpret_cast<uintptr_t>(htraj->no_break) & 7))
    return fail(hipErrorInvalidValue, "%s", "no_break must be 8-byte aligned");
  if ((traj->obs && (reinterpret_cast<uintptr_t>(traj->obs) & 15)) ||
      (traj->final_obs && (reinterpret_cast<uintptr_t>(traj->final_obs) & 7)) ||
      (traj->rew && (reinterpret_cast<uintptr_t>(traj->rew) & 7)) ||
      (reinterpret_cast<uintptr_t>(traj->flags) & 3))
    return fail(hipErrorInvalidValue, "%s", "traj.obs must be 16-byte, rew/final_obs 8-byte, flags 4-byte aligned");
  if (n == 0 || num_steps == 0) return 0;
  if (!(flags & MG_AUTORESET))  // hdqn.py's loop resets at every episode end (:276-277)
    return fail(hipErrorInvalidValue, "%s", "mg_rollout_hdqn needs MG_AUTORESET (hdqn.py resets every episode)");
  HRollout R{};
  R.P = *params;
  R.R0 = reset0(*params);
  R.S = *state;
  R.T = *traj;
  if (htraj) R.H = *htraj;
  if (stats) R.St = *stats;
  R.goal = goal;
  R.goal_op = goal_op;
  R.ext_acc = ext_acc;
  R.meta = static_cast<const uint8_t*>(meta_net);
  R.lower = static_cast<const uint8_t*>(lower_net);
  R.meta_op = static_cast<const uint8_t*>(opp_meta_net);
  R.lower_op = static_cast<const uint8_t*>(opp_lower_net);
  R.seed = seed;
  R.first_step = first_step;
  R.greedy_thr = greedy_threshold;
  R.env_offset = env_offset;
  R.n = n;
  R.num_steps = num_steps;
  R.num_goals = num_goals;
  R.reset_goal = reset_goal;
  R.flags = flags;
  R.ring = ring_rows;
  R.ring_counter = ring_counter;
  R.ring_capacity = ring_capacity;
  const unsigned blocks = static_cast<unsigned>((n + kHEnvs - 1) / kHEnvs);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (opponent_mode == 0)
    hipLaunchKernelGGL(hdqn_rollout_kernel<0>, dim3(blocks), dim3(512), 0, st, R);
  else if (opponent_mode == 1)
    hipLaunchKernelGGL(hdqn_rollout_kernel<1>, dim3(blocks), dim3(512), 0, st, R);
  else if (opponent_mode == 2)
    hipLaunchKernelGGL(hdqn_rollout_kernel<2>, dim3(blocks), dim3(512), 0, st, R);
  else
    hipLaunchKernelGGL(hdqn_rollout_kernel<3>, dim3(blocks), dim3(512), 0, st, R);
  if (ring_rows)  // after every block has read the old counter: the same stream orders it
    hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, st, ring_counter,
                       static_cast<uint64_t>(num_steps) * static_cast<uint64_t>(n));
  return finish_launch("mg_rollout_hdqn");
}

size_t mg_replay_scratch_bytes(int64_t n, int32_t num_steps) {
  if (n <= 0 || num_steps <= 0) return 0;
  const int64_t nb = ((n + kRBlock - 1) / kRBlock) * num_steps;
  const int64_t ng = replay_groups(nb);
  return static_cast<size_t>((8 + ng * 8 + nb * 4 + ng * 4 + 7) & ~int64_t{7});
}

int mg_replay_store(float* rows, uint64_t* counter, int64_t capacity, int32_t row_floats,
                    const mg_transitions* tr, int64_t n, int32_t num_steps, int32_t skip_ego_won,
                    void* scratch, size_t scratch_bytes, void* stream) {
  if (!rows || !counter || !tr) return fail(hipErrorInvalidValue, "%s", "mg_replay_store: NULL pointer");
  if (capacity < 1) return fail(hipErrorInvalidValue, "%s", "mg_replay_store: capacity < 1");
  if (row_floats != (tr->goal ? kRowGoal : kRow) || (tr->goal != nullptr) != (tr->next_goal != nullptr))
    return fail(hipErrorInvalidValue, "%s",
                "mg_replay_store: row_floats must be 22, or 24 with both goal and next_goal set");
  if (tr->meta_goal && (tr->goal || !tr->reward || !tr->won_mask))
    return fail(hipErrorInvalidValue, "%s",
                "mg_replay_store: meta_goal (Goal_DQN rows) needs reward and won_mask (no_break) and no goal");
  if (n < 0 || num_steps < 0) return fail(hipErrorInvalidValue, "%s", "mg_replay_store: n < 0 or num_steps < 0");
  if (n == 0 || num_steps == 0) return 0;
  if (!tr->obs_first || !tr->obs || !(tr->a1 || tr->flags) || !tr->rew)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_store: obs_first, obs, a1 (or flags) and rew are required");
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(tr->obs_first) |
       reinterpret_cast<uintptr_t>(tr->obs) | reinterpret_cast<uintptr_t>(tr->final_obs) |
       reinterpret_cast<uintptr_t>(tr->rew) | reinterpret_cast<uintptr_t>(scratch)) & 7)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_store: float buffers and scratch must be 8-byte aligned");
  if ((reinterpret_cast<uintptr_t>(tr->goal) | reinterpret_cast<uintptr_t>(tr->next_goal) |
       reinterpret_cast<uintptr_t>(tr->reward)) & 3)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_store: goal, next_goal and reward must be 4-byte aligned");
  const int64_t nbx = (n + kRBlock - 1) / kRBlock;
  const int64_t nb = nbx * num_steps;
  if (nbx > 0x7fffffff || replay_groups(nb) > 0x7fffffff)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_store: n * num_steps exceeds the grid limit");
  if (!scratch || scratch_bytes < mg_replay_scratch_bytes(n, num_steps))
    return fail(hipErrorInvalidValue, "%s", "mg_replay_store: scratch smaller than mg_replay_scratch_bytes(n, num_steps)");
  const unsigned chunks = static_cast<unsigned>((num_steps + kRTChunk - 1) / kRTChunk);
  if (chunks > 65535) return fail(hipErrorInvalidValue, "%s", "mg_replay_store: num_steps too large");
  ReplayIn R{};
  R.X = *tr;
  R.n = n;
  R.words = (n + 63) >> 6;
  R.nbx = nbx;
  R.nb = nb;
  R.T = num_steps;
  R.skip_won = tr->meta_goal ? 1 : skip_ego_won;  // Goal_DQN rows: keep the steps that broke
  const ReplayScratch S = replay_scratch(scratch, nb);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(replay_scan_kernel, dim3(static_cast<unsigned>(replay_groups(nb))), dim3(64), 0, st,
                     R, S);
  hipLaunchKernelGGL(replay_group_scan_kernel, dim3(1), dim3(64), 0, st, S, replay_groups(nb), counter);
  if (tr->goal)
    hipLaunchKernelGGL(replay_write_kernel<1>, dim3(static_cast<unsigned>(nbx), chunks), dim3(kRBlock), 0,
                       st, R, S, counter, rows, capacity);
  else if (tr->meta_goal)
    hipLaunchKernelGGL(replay_write_kernel<2>, dim3(static_cast<unsigned>(nbx), chunks), dim3(kRBlock), 0,
                       st, R, S, counter, rows, capacity);
  else
    hipLaunchKernelGGL(replay_write_kernel<0>, dim3(static_cast<unsigned>(nbx), chunks), dim3(kRBlock), 0,
                       st, R, S, counter, rows, capacity);
  return finish_launch("mg_replay_store");
}

int mg_replay_sample(const float* rows, const uint64_t* counter, int64_t capacity,
                     int32_t row_floats, uint64_t seed, uint64_t draw, int32_t filled_only,
                     float* out, int64_t* idx_out, int64_t batch, void* stream) {
  if (row_floats != kRow && row_floats != kRowGoal)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_sample: row_floats must be 22 or 24");
  if (!rows || !out || (filled_only && !counter))
    return fail(hipErrorInvalidValue, "%s", "mg_replay_sample: NULL pointer");
  if (capacity < 1 || capacity > (int64_t{1} << 32) || batch < 0)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_sample: need 1 <= capacity <= 2^32 and batch >= 0");
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(out)) & 7)
    return fail(hipErrorInvalidValue, "%s", "mg_replay_sample: rows and out must be 8-byte aligned");
  if (batch == 0) return 0;
  const unsigned blocks = static_cast<unsigned>((batch + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(replay_sample_kernel, dim3(blocks), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), rows, counter, capacity, row_floats, seed, draw,
                     filled_only, out, idx_out, batch);
  return finish_launch("mg_replay_sample");
}

int mg_reset(const mg_params* params, const mg_state* state, const uint8_t* mask,
             const mg_outputs* out, int64_t n, void* stream) {
  if (!params) return fail(hipErrorInvalidValue, "%s", "params is NULL");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (int e = check_state(state)) return e;
  if (n == 0) return 0;
  mg_outputs o{};
  if (out) o = *out;
  const unsigned blocks = static_cast<unsigned>((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(reset_kernel, dim3(blocks), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), *params, *state, mask, o, n);
  return finish_launch("mg_reset");
}

int mg_observe(const mg_params* params, const mg_state* state, const mg_outputs* out, int64_t n,
               void* stream) {
  if (int e = check_common(params, state, out, n)) return e;
  if (n == 0) return 0;
  const unsigned blocks = static_cast<unsigned>((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(observe_kernel, dim3(blocks), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), *params, *state, *out, n);
  return finish_launch("mg_observe");
}

size_t mg_stats_reduce_scratch_bytes(int64_t n) {
  if (n <= 0) return 0;
  return static_cast<size_t>((n + kRedEnvs - 1) / kRedEnvs) * sizeof(mg_stats_totals);
}

int mg_stats_reduce(const mg_episode_stats* rec, int64_t n, mg_stats_totals* totals, void* scratch,
                    size_t scratch_bytes, void* stream) {
  if (!totals || (n > 0 && !rec)) return fail(hipErrorInvalidValue, "%s", "mg_stats_reduce: NULL pointer");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (((reinterpret_cast<uintptr_t>(rec) | reinterpret_cast<uintptr_t>(scratch)) & 15) ||
      (reinterpret_cast<uintptr_t>(totals) & 7))
    return fail(hipErrorInvalidValue, "%s", "mg_stats_reduce: rec and scratch must be 16-byte, totals 8-byte aligned");
  const int64_t nb = (n + kRedEnvs - 1) / kRedEnvs;
  if (nb > 0x7fffffff) return fail(hipErrorInvalidValue, "%s", "n exceeds the grid limit");
  if (n > 0 && (!scratch || scratch_bytes < mg_stats_reduce_scratch_bytes(n)))
    return fail(hipErrorInvalidValue, "%s", "mg_stats_reduce: scratch smaller than mg_stats_reduce_scratch_bytes(n)");
  hipStream_t st = static_cast<hipStream_t>(stream);
  mg_stats_totals* part = static_cast<mg_stats_totals*>(scratch);
  if (nb > 0)
    hipLaunchKernelGGL(stats_reduce_kernel, dim3(static_cast<unsigned>(nb)), dim3(kRedThreads), 0, st, rec, n, part);
  hipLaunchKernelGGL(stats_reduce_final_kernel, dim3(1), dim3(kRedThreads), 0, st, part, nb, totals);
  return finish_launch("mg_stats_reduce");
}

int mg_host_step(const mg_params* params, const mg_state* state, const int8_t* a1, const int8_t* a2,
                 const mg_outputs* out, const mg_stats* stats, int64_t n, uint32_t flags) {
  if (int e = check_common(params, state, out, n)) return e;
  if (n == 0) return 0;
  if (!a1) return fail(hipErrorInvalidValue, "%s", "a1 is NULL");
  Launch L{};
  L.P = *params;
  L.R0 = reset0(*params);
  L.S = *state;
  L.O = *out;
  if (stats) L.St = *stats;
  L.a1 = a1;
  L.a2 = a2;
  L.n = n;
  L.flags = flags;
  for (int64_t w = 0; w < n; w += 64) {  // one 64-env group per done / won mask word
    uint64_t dm = 0, wm = 0;
    const int64_t end = n - w < 64 ? n : w + 64;
    for (int64_t i = w; i < end; ++i) {
      bool d, won;
      host_step_env(L, i, d, won);
      dm |= static_cast<uint64_t>(d) << (i - w);
      wm |= static_cast<uint64_t>(won) << (i - w);
    }
    if (L.O.done_mask) L.O.done_mask[w >> 6] = dm;
    if (L.O.won_mask) L.O.won_mask[w >> 6] = wm;
  }
  g_err[0] = '\0';
  return 0;
}

int mg_host_reset(const mg_params* params, const mg_state* state, const uint8_t* mask,
                  const mg_outputs* out, int64_t n) {
  if (!params) return fail(hipErrorInvalidValue, "%s", "params is NULL");
  if (n < 0) return fail(hipErrorInvalidValue, "%s", "n < 0");
  if (int e = check_state(state)) return e;
  mg_outputs o{};
  if (out) o = *out;
  for (int64_t i = 0; i < n; ++i)
    if (!mask || mask[i]) host_reset_env(*params, *state, o, i);
  g_err[0] = '\0';
  return 0;
}

int mg_host_observe(const mg_params* params, const mg_state* state, const mg_outputs* out, int64_t n) {
  if (int e = check_common(params, state, out, n)) return e;
  for (int64_t i = 0; i < n; ++i) host_observe_env(*params, *state, *out, i);
  g_err[0] = '\0';
  return 0;
}

}  // extern "C"
