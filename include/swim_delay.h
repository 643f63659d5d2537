/*
 * swim_delay.h — NetworkEmulator message delay quantised to engine ticks (specification).
 *
 * The reference delays every outbound message by floor(-ln(1 - x) * meanDelay) ms, x uniform in
 * [0, 1) (NetworkEmulator.evaluateDelay :359-369, applied by tryDelayOutbound :190-202 to every
 * send and requestResponse of NetworkEmulatorTransport :49-75).  The lockstep engine draws x from
 * the Philox hook (swim_rng.h) as a 53-bit integer u53 = (w0 >> 11) << 32 | w1 (the first two words
 * of the draw's block) and delivers the message floor(delay_ms / tick_ms) ticks after it was sent:
 *
 *   ticks(u53) = #{ j in [1, SWIM_DELAY_TICKS_MAX] : u53 >= TH_j },
 *   TH_j = ceil((1 - exp(-j * tick_ms / meanDelay)) * 2^53)        (UINT64_MAX once it reaches 2^53)
 *
 * which is floor(floor(-ln(1 - u53 / 2^53) * meanDelay) / tick_ms) with the comparison done on
 * integers.  The thresholds are computed once per distinct meanDelay on the host, by this one
 * function, in the GPU engine and in the CPU oracle alike (same libm at run time), so both engines
 * quantise every draw identically; the device and the oracle only compare integers.  Delays are
 * capped at SWIM_DELAY_TICKS_MAX ticks; a draw reaches the cap with probability
 * exp(-SWIM_DELAY_TICKS_MAX * tick_ms / meanDelay), so both engines refuse (SWIM_EINVAL) a mean
 * above SWIM_DELAY_MEAN_MAX_TICKS ticks (swim_delay_mean_ok): at the limit that probability is
 * e^-32 = 1.3e-14 per draw (at the reference's GossipDelayTest 3 s over 100 ms ticks, e^-68).
 */
#ifndef SWIM_DELAY_H
#define SWIM_DELAY_H

#include <math.h>
#include <stdint.h>

#define SWIM_DELAY_TICKS_MAX 2047u /* < the 2,048 arrival buckets of the GPU's delay ring */

#define SWIM_DELAY_MEAN_MAX_TICKS 64u /* SWIM_DELAY_TICKS_MAX / 64 = 32 means: cap probability e^-32 */

/* a meanDelay the tick-quantised delay can represent without truncating draws (mean_ms > 0) */
static inline int swim_delay_mean_ok(int32_t mean_ms, uint32_t tick_ms) {
  return mean_ms > 0 && (uint64_t)mean_ms <= (uint64_t)SWIM_DELAY_MEAN_MAX_TICKS * tick_ms;
}

static inline void swim_delay_thresholds(int32_t mean_ms, uint32_t tick_ms, uint64_t* th /* [SWIM_DELAY_TICKS_MAX] */) {
  for (uint32_t j = 1; j <= SWIM_DELAY_TICKS_MAX; ++j) {
    const double q = -expm1(-(double)j * (double)tick_ms / (double)mean_ms); /* P(x < ...) = 1 - e^-jt/M */
    const double s = ceil(ldexp(q, 53));
    th[j - 1] = s >= 9007199254740992.0 ? UINT64_MAX : (uint64_t)s;
  }
}

/* number of thresholds <= u53 (the thresholds ascend) */
#if defined(__HIPCC__)
__host__ __device__
#endif
static inline uint32_t swim_delay_ticks(const uint64_t* th, uint64_t u53) {
  uint32_t lo = 0, hi = SWIM_DELAY_TICKS_MAX;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (th[mid] <= u53) lo = mid + 1; else hi = mid;
  }
  return lo;
}

#endif
