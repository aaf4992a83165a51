// mc_fspec_f2.hip -- the speculative float Delta decode (mc_fspec.h) into
// little-endian f2; one translation unit per output dtype and byte order
// (mc_fspec_f2_be.hip) so that the instances build in parallel.
#include "mc_fspec.h"

void mc_fspec_launch_f2(const uint8_t *s, uint8_t *d, size_t n, int a, void *ws, uint32_t *ticket, hipStream_t st) {
  if (a == MC_F2) return launch_fspec<MC_F2, MC_F2>(s, d, n, a, ws, ticket, st);
  launch_fspec<-1, MC_F2>(s, d, n, a, ws, ticket, st);
}

void mc_fspec_rows_launch_f2(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a,
                              uint64_t *fail, unsigned g, hipStream_t st) {
  if (a == MC_F2) return launch_fspec_rows<MC_F2, MC_F2>(sc, ss, dc, ds, n, a, fail, g, st);
  launch_fspec_rows<-1, MC_F2>(sc, ss, dc, ds, n, a, fail, g, st);
}
