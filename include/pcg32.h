/* pcg32.h — drop-in for ray-tracing-c include/pcg32.h (reference include/pcg32.h:1-18).
 *
 * Permuted congruential generator (pcg-c-basic "pcg32"): 64-bit LCG state, XSH-RR 32-bit output.
 * The renderer seeds one generator per pixel as pcg32_seed(&g, 17 + row, 23 + col)
 * (reference src/raytracing.c:94) and the device kernel reproduces the exact same stream
 * (ray-tracing-c_amd/csrc/rt_device.h, rt_pcg32).
 */
#ifndef RT_PCG32_H
#define RT_PCG32_H
#ifndef PCG32_H
#define PCG32_H
#endif

#include <stdint.h>

typedef struct PCG32 {
  uint64_t state; /* LCG state, advanced by state * 6364136223846793005 + inc */
  uint64_t inc;   /* stream selector, always odd: (initseq << 1) | 1 */
} PCG32;

/* reference src/pcg32.c:3-9 */
void pcg32_seed(PCG32 *rng, uint64_t initstate, uint64_t initseq);
/* reference src/pcg32.c:11-17 */
uint32_t pcg32_u32(PCG32 *rng);
/* lo + u32 % (hi - lo); reference src/pcg32.c:18-20 */
uint32_t pcg32_u32_between(PCG32 *rng, uint32_t lo, uint32_t hi);
/* top 24 bits / 2^24 in [0,1); reference src/pcg32.c:21 */
float pcg32_f32(PCG32 *rng);
/* lo + f32 * (hi - lo); reference src/pcg32.c:22 */
float pcg32_f32_between(PCG32 *rng, float lo, float hi);

#endif /* RT_PCG32_H */
