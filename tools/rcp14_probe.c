/* Dumps the host CPU's VRCP14PD for every mantissa bucket (the top 16
 * fraction bits decide the result: tools/gen_np_math.py) as 65536 uint64,
 * probed at 1 + i/65536 + 2^-52 (bucket 0 then gives the value of every
 * input but the exact power of two, whose reciprocal is exact), then the
 * same 65536 probes at the bucket starts 1 + i/65536.
 *   gcc -O2 -mavx512f tools/rcp14_probe.c -o /tmp/rcp14_probe && /tmp/rcp14_probe out.bin */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(int argc, char** argv) {
  FILE* f = fopen(argc > 1 ? argv[1] : "rcp14_table.bin", "wb");
  if (!f) return 1;
  for (uint64_t low = 1;; low = 0) {
    for (uint32_t i = 0; i < 65536; i++) {
      uint64_t u = 0x3FF0000000000000ull | ((uint64_t)i << 36) | low, r;
      double x, o[8];
      memcpy(&x, &u, 8);
      _mm512_storeu_pd(o, _mm512_rcp14_pd(_mm512_set1_pd(x)));
      memcpy(&r, &o[0], 8);
      fwrite(&r, 8, 1, f);
    }
    if (!low) break;
  }
  return fclose(f) != 0;
}
