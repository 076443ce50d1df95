/*
 * kp_diag.h — measurement-variant knobs of csrc/kp_kernels.hip. TOOLS ONLY.
 *
 * The production build (karpenter-provider-aws_amd/Makefile) never includes this header and sets none of the knobs:
 * kp_kernels.hip refuses to compile when any of them is defined without KP_DIAG_BUILD, and static_asserts the
 * production values. tools/build_variant.sh and tools/build_fine.sh force-include this header (-include) and pass
 * their -D flags on top, into tools/variants/<name>/libkp.so or tools/fine/libkp.so (selected with KP_LIB=...).
 *
 * Knobs (production value in brackets):
 *   FASTLANE [1]         solve_kernel's wave-0 fast lane (0: full path only)
 *   FL_NOTIME [1]        fast-lane s_memtime phase probes compiled out (0: probes on, KP_TIMING reads them)
 *   FT_FINE [0]          finer fast-lane probes in place of the full path's attempt split
 *   FAST_SCAN_MAX [512]  longest first-fit scan the fast lane takes on
 *   FAST_CHK_LIVE [8]    chunked order: live chunks the fast lane scans before the 4-wave pre-pass
 *   FAST_EX_ROUNDS [8]   existing nodes: 64-position rounds the fast lane scans before the full path
 *   FAST_CONT [1]        the continuation round (the previous commit's NodeClaim first, from registers)
 *   SORT_DIAG [0]        the full path's sort split in stats[25..30]
 *   EX_DIAG [0]          the existing-node scan split in stats[25..30]
 *   FX_DIAG [0]          the fast lane's existing-node scans (scans, rounds, placed, skipped, failed, bailed) in stats[25..30]
 *   FEAS_MAX_BLOCKS [65536], FEASQ_EW [7], FEASQ_ROWS [28], FEASQ_B128 [1]  feasibility grid / block shape
 *   FEASQ_SKIP_EVAL [0]  decode + copies only, no type-set work: WRONG MASKS, timing experiments only
 *   FEASQ_MINW [6]       feasibility_quad_kernel register budget (waves per SIMD)
 *   SIM_WPE [0]          sim_kernel's register budget as waves per SIMD (amdgpu_waves_per_eu; 0: the compiler's)
 *   FL_SKIP [0]          fast-lane cost attribution, WRONG PLACEMENTS: bit 0 no sort replay, bit 1 no mutation stack,
 *                        bit 2 no statistics counters
 */
#pragma once
#define KP_DIAG_BUILD 1
