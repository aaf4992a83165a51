// mc_fspec_f8.hip -- the speculative float Delta decode (mc_fspec.h) into
// little-endian f8; one translation unit per output dtype and byte order
// (mc_fspec_f8_be.hip) so that the instances build in parallel.
#include "mc_fspec.h"

void mc_fspec_launch_f8(const uint8_t *s, uint8_t *d, size_t n, int a, void *ws, uint32_t *ticket, hipStream_t st) {
  if (a == MC_F8) return launch_fspec<MC_F8, MC_F8>(s, d, n, a, ws, ticket, st);
  if (a == MC_F4 && (uintptr_t)s % 8 == 0) return launch_fspec<MC_F4, MC_F8>(s, d, n, a, ws, ticket, st);
  launch_fspec<-1, MC_F8>(s, d, n, a, ws, ticket, st);
}

void mc_fspec_rows_launch_f8(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a,
                              uint64_t *fail, unsigned g, hipStream_t st) {
  if (a == MC_F8) return launch_fspec_rows<MC_F8, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
  if (a == MC_F4 && (uintptr_t)sc % 8 == 0 && ss % 8 == 0)
    return launch_fspec_rows<MC_F4, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
  launch_fspec_rows<-1, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
}
