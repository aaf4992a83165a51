// lab_sched.hip -- LAB ONLY: schedule overrides of the product kernels.
//
// libmcodec_lab.so links the product objects, so it owns a copy of their
// mc_sched (numcodecs_amd/csrc/mc_sched.h).  This file is the only place the
// MCODEC_* tuning variables are read: once when the lab library is loaded
// (so the sweep scripts under tools/ keep working when they point
// NUMCODECS_AMD_LIB at the lab library), and mc_lab_set_sched() changes a
// field by name at any time (tests/test_gpu_sched.py walks every alternative
// value against the oracle).  The product library reads no environment.
#include <stdlib.h>
#include <string.h>

#include "mc_common.h"

namespace {

struct field {
  const char *name;  // mc_lab_set_sched name
  const char *env;   // the MCODEC_* variable of the sweep scripts
  int *slot;
};

const field kFields[] = {
    {"copy_u", "MCODEC_COPY_U", &mc_sched.copy_u},
    {"copy_grid", "MCODEC_COPY_GRID", &mc_sched.copy_grid},
    {"ck_k", "MCODEC_CK_K", &mc_sched.ck_k},
    {"ck_kcopy", "MCODEC_CK_KCOPY", &mc_sched.ck_kcopy},
    {"ck_grid", "MCODEC_CK_GRID", &mc_sched.ck_grid},
    {"ck_grid_copy", "MCODEC_CK_GRID_COPY", &mc_sched.ck_grid_copy},
    {"f32_unroll", "MCODEC_F32_UNROLL", &mc_sched.f32_unroll},
    {"f32_ntld", "MCODEC_F32_NTLD", &mc_sched.f32_ntld},
    {"f32_fused_grid", "MCODEC_F32_FUSED_GRID", &mc_sched.f32_fused_grid},
    {"f32_slice_kb", "MCODEC_F32_SLICE_KB", &mc_sched.f32_slice_kb},
    {"c4_group_mi", "MCODEC_C4_GROUP_MI", &mc_sched.c4_group_mi},
    {"delta_enc_vec", "MCODEC_DELTA_ENC_VEC", &mc_sched.delta_enc_vec},
    {"dscan", "MCODEC_DSCAN", &mc_sched.dscan},
    {"dscan_nt", "MCODEC_DSCAN_NT", &mc_sched.dscan_nt},
    {"fspec", "MCODEC_FSPEC", &mc_sched.fspec},
    {"fastdiv", "MCODEC_FASTDIV", &mc_sched.fastdiv},
    {"crc_lds", "MCODEC_CRC_LDS", &mc_sched.crc_lds},
    {"delta_enc_dv", "MCODEC_DELTA_ENC_DV", &mc_sched.delta_enc_dv},
    {"br_planes", "MCODEC_BR_PLANES", &mc_sched.br_planes},
    {"ck_fused_plain", "MCODEC_CK_FUSED_PLAIN", &mc_sched.ck_fused_plain},
};

__attribute__((constructor)) void lab_sched_from_env() {
  for (const field &f : kFields) {
    const char *v = getenv(f.env);
    if (v && *v) *f.slot = atoi(v);
  }
}

}  // namespace

extern "C" {

// Set schedule field `name`; returns the previous value, or INT32_MIN for an
// unknown name.
int mc_lab_set_sched(const char *name, int value) {
  for (const field &f : kFields)
    if (!strcmp(f.name, name)) {
      const int old = *f.slot;
      *f.slot = value;
      return old;
    }
  return INT32_MIN;
}

int mc_lab_get_sched(const char *name) {
  for (const field &f : kFields)
    if (!strcmp(f.name, name)) return *f.slot;
  return INT32_MIN;
}

}  // extern "C"
