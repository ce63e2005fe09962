// sl_rollout.hip -- the per-step arithmetic of the PPO caller, on the device.
//
//   sl_sample_actions   np.random.choice(len(policy), p=policy) for every env
//                       (training/ppo.py:440; numpy's legacy RandomState.choice)
//   sl_gae              discounted returns + GAE advantages over a [T, N] rollout
//                       (training/ppo.py:487-503)
//
// Both are tiny HBM-bound passes next to the env step: one thread per env (sampling,
// reads A probabilities) or per (env, discount) column (GAE, a reverse scan over T
// whose loads are coalesced across envs at every t).  The float rounding follows the
// reference's numpy dtypes step by step (float32 policy/values/gamma, float64
// rewards), and the library is built with -ffp-contract=off, so results are
// bit-identical to the numpy expressions they restate.
#include "sl_device.h"
#include "../../include/safelife_hip.h"

using namespace sl;

namespace {

constexpr int NT = 256;
constexpr uint32_t kActionTensor = 2;     // Philox counter c3 of action draws
                                          // (0/1: board/goals spawns, 4/5: rollouts)

// numpy.random.RandomState.choice(a, p=p) with a = A, size = None:
//   p is converted to float64; p < 0 anywhere -> ValueError; |kahan_sum(p) - 1| > atol
//   -> ValueError; cdf = cumsum(p); cdf /= cdf[-1]; u = random_sample();
//   idx = cdf.searchsorted(u, side='right')  (= #{k : cdf[k] <= u}).
template <typename P>
__global__ void __launch_bounds__(NT)
k_sample_actions(const P *__restrict__ probs, int64_t B, int A, int64_t ld, int rng_mode,
                 const double *__restrict__ u_in, uint64_t seed, uint32_t env0, uint32_t step,
                 double atol, int32_t *__restrict__ actions, uint8_t *__restrict__ err) {
    const int64_t b = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (b >= B) return;
    const P *p = probs + b * ld;
    double cdf = 0.0, ks = (double)p[0], kc = 0.0;
    bool neg = false;
    for (int k = 0; k < A; k++) {
        const double v = (double)p[k];
        neg |= v < 0.0;
        cdf = cdf + v;
        if (k > 0) {                      // kahan_sum (numpy/random/_common.pyx)
            const double y = v - kc;
            const double t = ks + y;
            kc = (t - ks) - y;
            ks = t;
        }
    }
    const double total = cdf;
    const double u = rng_mode == SL_RNG_STREAM
                         ? u_in[b]
                         : philox_uniform(0u, env0 + (uint32_t)b, step, kActionTensor, seed);
    int idx = 0;
    double c = 0.0;
    for (int k = 0; k < A; k++) {
        c = c + (double)p[k];
        idx += (c / total <= u) ? 1 : 0;
    }
    actions[b] = idx;
    if (err) err[b] = (uint8_t)((neg ? 1 : 0) | (fabs(ks - 1.0) > atol ? 2 : 0));
}

// One (env n, discount g) column of gen_training_batch (ppo.py:487-503):
//   r = clip(rewards) (float64); m = ~end_episode
//   advantages = r + (gamma * m * values[1:]) [float32] - values[:-1]
//   returns[-1] = r[-1] + (m[-1] * gamma * values[-1]) [float32]
//   returns[i] = r[i] + (gamma * m[i]) [float32] * returns[i+1]
//   advantages[i] += (lmda * m[i]) [float32] * advantages[i+1]
__global__ void __launch_bounds__(NT)
k_gae(const double *__restrict__ rewards, const uint8_t *__restrict__ dones,
      const float *__restrict__ values, const float *__restrict__ gamma,
      const float *__restrict__ lmda, int G, int T, int64_t N, double clip,
      double *__restrict__ returns, double *__restrict__ adv) {
    const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (j >= N * G) return;
    const int64_t n = j / G;
    const int g = (int)(j - n * G);
    const float gm = gamma[g], lm = lmda[g];
    const int64_t NG = N * G;
    double ret_next = 0.0, adv_next = 0.0;
    for (int t = T - 1; t >= 0; t--) {
        double r = rewards[t * N + n];
        if (clip > 0.0) r = fmin(fmax(r, -clip), clip);
        const bool m = dones[t * N + n] == 0;
        const float v0 = values[t * NG + j], v1 = values[(t + 1) * NG + j];
        const float gmask = m ? gm : 0.0f;            // gamma * reward_mask (float32)
        const float lmask = m ? lm : 0.0f;            // lmda * reward_mask
        double a = (r + (double)(gmask * v1)) - (double)v0;
        double ret;
        if (t == T - 1) {
            ret = r + (double)(gmask * v1);
        } else {
            ret = r + (double)gmask * ret_next;
            a = a + (double)lmask * adv_next;
        }
        returns[t * NG + j] = ret;
        adv[t * NG + j] = a;
        ret_next = ret;
        adv_next = a;
    }
}

unsigned blocks(int64_t n) { return (unsigned)((n + NT - 1) / NT); }

}  // namespace

extern "C" int sl_sample_actions(const void *probs, int probs_f64, int64_t B, int A,
                                 int64_t ld, int rng_mode, const double *uniforms,
                                 uint64_t seed, uint32_t env0, uint32_t step, double atol,
                                 int32_t *actions, uint8_t *err, void *stream) {
    if (B < 0 || A < 1 || ld < A || !probs || !actions) return SL_EINVAL;
    if (rng_mode == SL_RNG_STREAM && !uniforms) return SL_EINVAL;
    if (rng_mode != SL_RNG_STREAM && rng_mode != SL_RNG_PHILOX) return SL_EINVAL;
    if (B == 0) return SL_OK;
    hipStream_t s = (hipStream_t)stream;
    if (probs_f64)
        k_sample_actions<double><<<blocks(B), NT, 0, s>>>(
            (const double *)probs, B, A, ld, rng_mode, uniforms, seed, env0, step, atol,
            actions, err);
    else
        k_sample_actions<float><<<blocks(B), NT, 0, s>>>(
            (const float *)probs, B, A, ld, rng_mode, uniforms, seed, env0, step, atol,
            actions, err);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_gae(const double *rewards, const uint8_t *end_episode, const float *values,
                      const float *gamma, const float *lmda, int G, int T, int64_t N,
                      double reward_clip, double *returns, double *advantages, void *stream) {
    if (G < 1 || T < 1 || N < 0 || !rewards || !end_episode || !values || !gamma || !lmda ||
        !returns || !advantages)
        return SL_EINVAL;
    if (N == 0) return SL_OK;
    k_gae<<<blocks(N * G), NT, 0, (hipStream_t)stream>>>(rewards, end_episode, values, gamma,
                                                          lmda, G, T, N, reward_clip, returns,
                                                          advantages);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}
