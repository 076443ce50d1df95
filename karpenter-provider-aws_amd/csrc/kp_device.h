// kp_device.h — kernel argument blocks (host <-> device), plain pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_model.h"

struct SolveArgs {
  const DevDict* dict;
  const DevCatalog* cats;
  int32_t n_catalogs;
  const int64_t* vint;  // [W*64]
  // pods
  int32_t n_pods;
  const int32_t* pod_shape;      // [P]
  int32_t* pod_level;            // [P] relaxation level (mutable)
  int32_t* queue;                // [P] ring, pre-sorted byCPUAndMemoryDescending
  int32_t* lastlen;              // [P]
  int32_t* lastlen_epoch;        // [P]
  // shapes (x relaxation levels)
  const int32_t* shape_level_base;   // [S]
  const int32_t* shape_nlevels;      // [S]
  const uint8_t* shape_reqs;         // [SL] KReqs
  const uint64_t* shape_negop;       // [SL]
  const int64_t* shape_requests;     // [S][NRES]
  const uint64_t* shape_tolerates;   // [S] bit ts: tolerates taint set ts
  const uint64_t* shape_pvp;         // rows of TW words
  const int32_t* pvp_base;           // [SL][n_catalogs] first row
  const int32_t* pvp_slot;           // [SL][64] row offset of key k (relative to base)
  // templates
  int32_t n_tmpl;
  const uint8_t* tmpl_reqs;          // [NT] KReqs
  const int32_t* tmpl_taintset;      // [NT]
  const int32_t* tmpl_catalog;       // [NT]
  const uint64_t* tmpl_X;            // [NT][TW] InstanceTypeOptions after NewScheduler's pre-filter
  const int64_t* tmpl_daemon;        // [NT][NRES]
  const uint32_t* tmpl_limit_present;// [NT]
  int64_t* tmpl_remaining;           // [NT][NRES] (mutable)
  // existing nodes (upstream order)
  int32_t n_existing;
  uint8_t* ex_reqs;                  // [E] KReqs (mutable)
  const int32_t* ex_taintset;        // [E]
  const int64_t* ex_available;       // [E][NRES]
  int64_t* ex_requests;              // [E][NRES] (mutable)
  // in-flight NodeClaims (capacity n_pods)
  uint8_t* nc_reqs;                  // [P] KReqs
  uint64_t* nc_X;                    // [P][TW]
  int64_t* nc_requests;              // [P][NRES]
  int32_t* nc_tmpl;                  // [P]
  int32_t* g_npods;                  // [P] len(Pods)
  int32_t* g_order;                  // [P] newNodeClaims order
  int32_t sort_in_lds;               // unused (LDS until SORT_CAP NodeClaims, then global)
  int32_t sort_cap;
  // exact failure memo: outcome of Add/CanAdd depends only on (candidate state, pod shape-level), so a
  // recorded failure stays valid while the candidate's version is unchanged
  int32_t ncc;                       // NodeClaim ids < ncc are memoised
  int32_t* nc_ver;                   // [P]
  int32_t* nc_fail;                  // [SL][ncc]
  int32_t* ex_ver;                   // [E]
  int32_t* ex_fail;                  // [SL][E]
  int32_t* tmpl_ver;                 // [NT]
  int32_t* tmpl_fail;                // [SL][NT]
  int64_t* nc_maxalloc;              // [P][NRES] max allocatable over the NodeClaim's types at creation
  int32_t* nc_fitj;                  // [P][NRES] threshold index of the last Fits per resource
  int32_t* nc_taintset;              // [P] taint set of the NodeClaim's template
  uint32_t req_res_mask;             // resources some pod shape requests (> 0)
  int32_t timing;                    // 1: thread 0 accumulates per-phase s_memtime deltas into stats[8..15]
  // outputs
  int32_t* placement;                // [P]
  int32_t* events;                   // [P] pods in placement order
  uint64_t* stats;                   // [8]: attempts, bytes, pops, n_nc, n_events
};

struct FinalizeArgs {
  const DevDict* dict;
  const DevCatalog* cats;
  const int64_t* vint;
  int32_t n_nc;
  const int32_t* nc_tmpl;
  const int32_t* tmpl_catalog;
  const uint8_t* nc_reqs;
  const uint64_t* nc_X;
  int32_t max_types;
  int32_t opt_stride;
  uint32_t* out_options;     // [n_nc][opt_stride]
  uint32_t* out_n_remaining; // [n_nc]
  uint32_t* out_n_options;   // [n_nc]
};

struct FeasArgs {
  const DevDict* dict;
  const DevCatalog* cat;
  const int64_t* vint;
  int32_t T;
  int32_t n_queries;
  int32_t mode_compatible;   // 1: Compatible(q, type, WK) (CompatibleAvailableFilter); 0: type.Intersects(q)
  int32_t pad_;
  const uint8_t* q_reqs;     // [Q] KReqs
  const int64_t* q_requests; // [Q][NRES]
  uint64_t* out_mask;        // [Q][tiles]
  double* out_cheapest;      // [Q][T] or null
};

hipError_t launch_solve(const SolveArgs& a, int nw, size_t dyn_lds, hipStream_t s);
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s);
hipError_t launch_feasibility(const FeasArgs& a, hipStream_t s);
