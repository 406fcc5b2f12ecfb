/* rt_turn_table.h -- the render kernel's sin/cos table:
 * (cos, sin)(2 pi i / RT_TURN_TABLE) for i < RT_TURN_TABLE, as fp32 pairs.
 * Computed with a Taylor series in IEEE double arithmetic (no libm, so every
 * compiler and C library gives the same bits) on the quadrant-reduced angle,
 * then rounded once to fp32 and mapped to its quadrant exactly.  The library
 * uploads it to each device; the oracle's kernel-mode restatement builds the
 * same table from this header. */
#ifndef RTOW_RT_TURN_TABLE_H
#define RTOW_RT_TURN_TABLE_H

#define RT_TURN_TABLE 1024

static inline void rt_turn_table(float *cos_sin /* 2 * RT_TURN_TABLE */) {
  const int n = RT_TURN_TABLE, q4 = RT_TURN_TABLE / 4;
  for (int i = 0; i < n; ++i) {
    const double x = 6.283185307179586476925 * (double)(i % q4) / (double)n; /* in [0, pi/2) */
    double c = 0.0, s = 0.0, term = 1.0; /* term = x^k / k! */
    for (int k = 0; k < 32; ++k) {
      switch (k % 4) {
        case 0: c += term; break;
        case 1: s += term; break;
        case 2: c -= term; break;
        default: s -= term; break;
      }
      term = term * x / (double)(k + 1);
    }
    const float fc = (float)c, fs = (float)s;
    float *o = cos_sin + 2 * i;
    switch (i / q4) {
      case 0: o[0] = fc; o[1] = fs; break;
      case 1: o[0] = -fs; o[1] = fc; break;
      case 2: o[0] = -fc; o[1] = -fs; break;
      default: o[0] = fs; o[1] = -fc; break;
    }
  }
}

#endif /* RTOW_RT_TURN_TABLE_H */
