// mc_sched.h -- schedule parameters of the product kernels.
//
// Every value below is the measured default documented where it is used (the
// sweeps that chose it are under profiles/).  The product library never
// changes them and reads no environment variable: a schedule cannot be
// switched behind the caller's back.  The lab library (tools/lab), which
// links the product objects, overrides fields for its sweeps and A/B runs
// (tools/lab/lab_sched.hip: MCODEC_* variables read at load time, and
// mc_lab_set_sched), and tests/test_gpu_sched.py checks every alternative
// value against the oracle through it.
#pragma once

struct mc_sched_t {
  int copy_u;          // mc_copy: 16-B vectors per thread per tile (4 or 8)
  int copy_grid;       // mc_copy: workgroup cap, 0 = one tile per workgroup
  int ck_k;            // checksum-only passes: tile = ck_k x 4 KiB (4, 8, 16; 0 = per-pass default)
  int ck_kcopy;        // copying checksum passes: tile = ck_kcopy x 4 KiB (4, 8, 16)
  int ck_grid;         // checksum-only grid cap, 0 = per-kind default
  int ck_grid_copy;    // copying checksum passes' grid cap
  int f32_unroll;      // Fletcher32 vectors in flight (1, 4, 8), 0 = per-pass default
  int f32_ntld;        // Fletcher32 nontemporal loads (0/1)
  int f32_fused_grid;  // one-launch Fletcher32 verify block cap (256 .. 65536)
  int f32_slice_kb;    // Fletcher32 payload KiB per workgroup (4 .. 4096)
  int c4_group_mi;     // batched C4 segment passes: Mi elements per group
  int delta_enc_vec;   // same-width integer Delta encode on the vector kernel (0/1)
  int dscan;           // same-width integer Delta decode on the k_dscan kernels (0/1)
  int dscan_nt;        // k_dscan two-launch decode: bit 0 nt reduce loads, bit 1 nt apply loads
  int fspec;           // speculative float Delta decode (0 = serial chain only)
  int fastdiv;         // FSO decode divides by the constant scale with the Markstein rcp (0/1)
  int crc_lds;         // CRC32/CRC32C tiles of >= 4 vectors per lane fold with the LDS slicing-by-16 tables (1) or bit-sliced XORs (0)
  int delta_enc_dv;    // same-type Delta encode (k_delta_enc_same): 16-B vectors per thread (4 or 8)
  int br_planes;       // BitRound+Shuffle(4) of one large chunk masks the planes (k_bitround_shuffle4_planes) (0/1)
  int ck_fused_plain;  // one-launch CRC encode to a 16-B aligned destination: plain (1) or nontemporal (0) 16-B stores
};

extern mc_sched_t mc_sched __attribute__((visibility("hidden")));
