// mc_fspec_f4_be.hip -- the speculative float Delta decode (mc_fspec.h)
// with a big-endian astype and/or output dtype f4: both big-endian and
// equal -> the constant-dtype instance (SW = 3, bytes reversed in registers
// after the vector loads / before the stores); otherwise the runtime-astype
// instance (a flagged astype is read through mc_num_from_bits), SW = 2 for a
// big-endian output.
#include "mc_fspec.h"

void mc_fspec_launch_be_f4(const uint8_t *s, uint8_t *d, size_t n, int a, bool swo, void *ws, uint32_t *ticket, hipStream_t st) {
  if (swo && a == (MC_F4 | MC_BIG_ENDIAN)) launch_fspec<MC_F4, MC_F4, 3>(s, d, n, a, ws, ticket, st);
  else if (swo) launch_fspec<-1, MC_F4, 2>(s, d, n, a, ws, ticket, st);
  else mc_fspec_launch_f4(s, d, n, a, ws, ticket, st);  // flagged a != MC_F4: the runtime-astype instance
}

void mc_fspec_rows_launch_be_f4(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a, bool swo,
                                 uint64_t *fail, unsigned g, hipStream_t st) {
  if (swo && a == (MC_F4 | MC_BIG_ENDIAN)) launch_fspec_rows<MC_F4, MC_F4, 3>(sc, ss, dc, ds, n, a, fail, g, st);
  else if (swo) launch_fspec_rows<-1, MC_F4, 2>(sc, ss, dc, ds, n, a, fail, g, st);
  else mc_fspec_rows_launch_f4(sc, ss, dc, ds, n, a, fail, g, st);
}
