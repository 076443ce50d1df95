// kp_device.h — kernel argument blocks (host <-> device), plain pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_model.h"

#define KP_SOLVE_STATS 48
// why the fast lane handed a popped pod to the full path (stats[32 + FB_*])
enum { FB_INELIGIBLE = 0, FB_SPILLED = 1, FB_SHIFT = 2, FB_SCAN = 3, FB_MERGE = 4, FB_MINVALUES = 5, FB_NONE = 6, FB_MEMO = 7 };

// The in-flight pre-check's view of one NodeClaim in one 64-byte line (one gather per candidate position instead of
// one per field): headroom = max allocatable over its types at creation minus its requests, for the first four
// requested resources (req_res_mask bit order; more are checked from nc_requests / nc_maxalloc), the exact failure
// memo's version, the taint set of its template.
struct NcHead {
  int64_t room[4];
  int32_t ver, taintset;
  int32_t pad_[6];
};

// One chunk of the spilled newNodeClaims order (solve_kernel's chunked mode): up to 64 NodeClaim ids in sorted order
// and their len(Pods).
struct ChkBlk {
  int32_t id[64];
  int32_t key[64];
};
#define CHK_MAXC 4096  // chunks (and blocks) of the chunked order; its directory lives in LDS
#define CHK_LDS_BYTES (CHK_MAXC * 14)  // the directory: start, info, block epochs (4 B each), free list (2 B)

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
  const uint64_t* shape_tolerates;   // [SL] bit ts: tolerates taint set ts (per level: toleratePreferNoScheduleTaints)
  const uint64_t* shape_pvp;         // rows of TW words
  const int32_t* pvp_base;           // [SL][n_catalogs] first row
  const int32_t* pvp_slot;           // [SL][64] row offset of key k (relative to base)
  const int32_t* sl_pvp_n;           // [SL] PVP rows of catalogue 0
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
  // batched simulations: the existing nodes' requirements copy-on-write. ex_reqs_ro = the pristine [E] KReqs (shared by
  // every simulation), ex_own = [ceil(E/64)] bits, set once the simulation wrote its own copy into ex_reqs (store_merged
  // writes a complete set: no copy first). ex_reqs_ro null: ex_reqs is complete (single Solves restore it per run).
  const uint8_t* ex_reqs_ro;
  uint64_t* ex_own;
  // batched simulations: per shape-level the existing positions that can ever pass its count-independent checks
  // (headroom, taints, static check, host ports on the superset's pristine state; nodes only fill up and a simulation
  // only excludes nodes), ascending: ex_ulist[ex_ulist_off[sl] .. ex_ulist_off[sl + 1]), and ex_uidx[sl][e] = the first
  // list index whose position is >= e. The full path's addToExistingNode scans the list instead of every position.
  // Null: scan every position.
  const int32_t* ex_ulist;
  const int32_t* ex_ulist_off;
  const int32_t* ex_uidx;
  const int32_t* ex_taintset;        // [E]
  const int64_t* ex_available;       // [E][NRES]
  int64_t* ex_requests;              // [E][NRES] (mutable)
  int64_t* ex_room;                  // [4][E] available - requests of the first four requested resources (mutable;
                                     // INT64_MAX past the requested ones)
  // in-flight NodeClaims (capacity n_pods)
  uint8_t* nc_reqs;                  // [P] KReqs
  uint64_t* nc_X;                    // [P][TW]
  int64_t* nc_requests;              // [P][NRES]
  int32_t* nc_tmpl;                  // [P]
  int32_t* g_npods;                  // [P] len(Pods)
  int32_t* g_order;                  // [P] newNodeClaims order
  int32_t sort_in_lds;               // unused (LDS until SORT_CAP NodeClaims, then global)
  int32_t sort_cap;
  // past sort_cap NodeClaims the order is chunked (chk_blk, directory in LDS); when the directory is full (or
  // chk_maxc == 0) it falls back to the flat global arrays g_order / g_npods
  ChkBlk* chk_blk;                   // [CHK_MAXC]
  int32_t* chk_dead;                 // [chk_dead_rows][CHK_MAXC] per (shape-level, block): the block's insertion epoch
                                     // when every NodeClaim in it failed the shape-level permanently (-1 none)
  int32_t chk_dead_rows;             // shape-levels < this keep dead marks
  int32_t chk_maxc;                  // chunks the directory may use (<= CHK_MAXC; a test hook lowers it)
  // exact failure memo: outcome of Add/CanAdd depends only on (candidate state, pod shape-level), so a
  // recorded failure stays valid while the candidate's version is unchanged
  int32_t ncc;                       // NodeClaim ids < ncc are memoised
  NcHead* nc_head;                   // [P] pre-check record (version, taint set, headroom), written at creation
  int32_t* nc_fail;                  // [SL][ncc]
  int32_t* ex_ver;                   // [E]
  int32_t* ex_fail;                  // [SL][E]
  int32_t* tmpl_ver;                 // [NT] bumped when the template's remaining limits change (subtractMax)
  int32_t* tmpl_fail;                // [SL][NT] NC_NEVER: the template fails the shape-level for good
  uint64_t* tmpl_xlim;               // [NT][TW] the template's options after filterByRemainingResources ...
  int32_t* tmpl_xlim_ver;            // [NT] ... as of this tmpl_ver (-1: never computed)
  int64_t* nc_maxalloc;              // [P][NRES] max allocatable over the NodeClaim's types at creation
  int32_t* nc_fitj;                  // [P][NRES] threshold index of the last Fits per resource
  int32_t* nc_cat;                   // [P] catalogue of the NodeClaim's template
  uint32_t req_res_mask;             // resources some pod shape requests (> 0)
  int32_t timing;                    // 1: thread 0 accumulates per-phase s_memtime deltas into stats[8..15]
  int32_t stop_nc;                   // > 0 (consolidation simulations): end the Solve once this many NodeClaims exist
  const int32_t* cancel;             // kp_cancel flag (host-mapped, polled every ~1024 pops), NULL: none
  int32_t cont;                      // 1: the fast lane variant with the continuation round (queue runs of one shape)
  // topology spread (upstream Topology, TopologyTypeSpread groups). A group on a dictionary key keeps a
  // count per value ordinal and the mask of registered domains; a hostname group a saturating u8 count per
  // node (existing positions: hcnt_ex, NodeClaim ids: hcnt_nc).
  int32_t n_groups;
  const int32_t* tg_key;             // [G] dictionary key, -1: hostname
  const int32_t* tg_row;             // [G] row of a hostname group in hcnt_*, -1 otherwise
  const int32_t* tg_maxskew;         // [G]
  const int32_t* tg_mindom;          // [G] minDomains, 0: nil
  const int32_t* tg_aff;             // [G] node filter has an affinity term (NodeAffinityPolicy Honor)
  const int32_t* tg_term_base;       // [G] its first term in tg_terms
  const int32_t* tg_nterm;           // [G] its terms (ORed: MakeTopologyNodeFilter over the required terms)
  int32_t* tg_live;                  // [G] 1: the group exists (mutable: a relaxation's Topology.Update makes it)
  const uint64_t* tg_filt_tol;       // [G] bit ts: node filter admits taint set ts (NodeTaintsPolicy)
  const uint8_t* tg_terms;           // KReqs
  const uint64_t* tg_terms_negop;
  int32_t* tg_cnt;                   // [G][64] (mutable)
  uint64_t* tg_reg;                  // [G] (mutable)
  uint8_t* hcnt_ex;                  // [GH][E] (mutable)
  uint8_t* hcnt_nc;                  // [GH][hnc_stride] (zeroed per run)
  int32_t hnc_stride;
  const int32_t* shape_rec_base;     // [S] groups that select the shape's pods (Topology.Record)
  const int32_t* shape_rec_n;        // [S]
  const int32_t* rec_list;
  const int32_t* sl_own_base;        // [SL] groups the shape-level owns (AddRequirements)
  const int32_t* sl_own_n;           // [SL] (<= 8)
  const int32_t* own_group;
  const int32_t* own_self;           // the group's selector matches the owner pod
  const uint64_t* own_pd;            // podDomains (strict requirements) over the key's value ordinals
  const int32_t* rec_aux;            // per rec_list entry: hostname row, else -1 - key slot (static)
  const int32_t* sl_fast_topo;       // [SL] 1: the fast lane may place the level's pods
  const int4* own_rec;               // [O][2] group, self, key, maxSkew | minDomains, row, key slot, 0 (static)
  const uint64_t* sl_topo_keys;      // [SL] dictionary keys of the owned groups
  const int32_t* sl_stage;           // [SL][64] the fast lane's stage record (topology Solves; kp_host StageRecords)
  // first-fit cursors (exact): cur_*[sl] = {k, t}: the first k candidates of the scan order were known to
  // fail for shape-level sl at mutation time t; a mutation stack (t, position, in LDS) clamps k to the lowest
  // position changed since (monotone stack: suffix minimum by binary search). Shape-levels that own
  // topology groups do not use them (their outcome depends on the counts).
  int32_t* cur_nc;                   // [SL][2] in-flight NodeClaims (positions in the sorted order)
  int32_t* cur_ex;                   // [SL][2] existing nodes (upstream order)
  // [SL] unschedulable memo: the NodeClaim count when a pod of the shape-level last failed every placement (-1:
  // never). Without topology or reservations and with no positive custom key at the level, every failure is
  // permanent (existing nodes and NodeClaims only fill up and narrow, limits only shrink as NodeClaims are created),
  // so a later pod of the level fails again exactly while no NodeClaim was created since
  int32_t* sl_fail;
  int32_t n_tk;                      // topology keys (dictionary keys some group spreads over)
  const int32_t* tk_keys;            // [TK]
  uint8_t* nc_tcode;                 // [TK][hnc_stride] pinned value ordinal per NodeClaim (store_tcodes)
  const uint8_t* ex_static_ok;       // [E] every unrequested resource fits and nothing available is negative
  int32_t n_req_res;                 // popcount(req_res_mask)
  const int32_t* tkey_slot;          // [64] row of a topology key in ex_tcode
  const uint8_t* ex_tcode;           // [TK][E] value ordinal of the existing node's label (0xFF: none)
  // host ports (upstream HostPortUsage, one bit per distinct port entry of the batch): a candidate conflicts when
  // its used bits meet the pod's conflict mask; a placement ORs in the pod's add mask (used bits only grow)
  int32_t hp_any;                    // some shape or existing node names a host port
  const uint64_t* shape_hp_conf;     // [S]
  const uint64_t* shape_hp_add;      // [S]
  uint64_t* ex_hp;                   // [E] (mutable)
  uint64_t* nc_hp;                   // [P] set when the NodeClaim is created
  // precomputed template options per (shape-level, template) (tmpl_feas_kernel), or null
  const uint64_t* tfeas;             // [SL][NT] entries of tfeas_words
  int32_t tfeas_words;
  // outputs
  int32_t* placement;                // [P]
  int32_t* events;                   // [P] pods in placement order
  uint64_t* stats;                   // [KP_SOLVE_STATS]: attempts, bytes, pops, n_nc, n_events, scanned, starts; [7] runaway;
                                     // [8..15] phases, [16..23] attempt split, [24] fast-lane pods, [25..30] fast-lane
                                     // cycles, [31] literal pdqsorts, [32..39] fast-lane hand-offs by reason (FB_*),
                                     // [40] pops whose addToNewNodeClaim failed on a ReservedOfferingError
  // capacity reservations (upstream ReservationManager + NodeClaim.reserveOfferings): res_mode 0 none, 1 fallback,
  // 2 strict. A reservation id is one offering class (res_cls); its remaining capacity lives in LDS during the Solve,
  // starting from res_cap0; nc_held[nc] = the classes NodeClaim nc holds (zeroed per run)
  int32_t res_mode;
  int32_t res_pad_;
  uint64_t res_cls;
  uint64_t* nc_held;                 // [P]
  int32_t res_cap0[KP_MAX_CLASSES];
};

// tmpl_feas_kernel: rows [row_lo, row_hi) of shape-levels x every template
struct TfeasArgs {
  const DevDict* dict;
  const DevCatalog* cats;
  int32_t n_catalogs;
  const int64_t* vint;
  int32_t n_tmpl;
  const uint8_t* tmpl_reqs;
  const int32_t* tmpl_catalog;
  const uint64_t* tmpl_X;
  const int64_t* tmpl_daemon;
  const uint8_t* shape_reqs;         // [SL] KReqs
  const uint64_t* shape_negop;       // [SL]
  const int32_t* sl_shape;           // [SL] shape of the shape-level
  const int64_t* shape_requests;     // [S][NRES]
  const uint64_t* shape_pvp;
  const int32_t* pvp_base;
  const int32_t* pvp_slot;
  const int32_t* sl_own_n;
  uint32_t req_res_mask;
  int32_t row_lo, row_hi;
  int32_t words;                     // u64 per entry: TW + KP_NRES / 2 + 1
  uint64_t* out;                     // [SL][NT] entries (this call writes rows [row_lo, row_hi))
};
hipError_t launch_tmpl_feas(const TfeasArgs& a, hipStream_t s);

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
  const uint64_t* nc_held;   // [n_nc] reservation classes held (FinalizeScheduling: reservation-id In {..}), or null
  const uint64_t* solve_stats;  // batched finalize: the Solve's stats (n_nc = [3]); unused otherwise
};

// batch_init_kernel: per-arena initialisation of batched Solves (pristine copy + byte fills)
constexpr int BATCH_INIT_FILLS = 12;
struct BatchInitArgs {
  uint8_t* base;
  size_t stride;
  const uint8_t* pristine;
  size_t dst_off, n_copy;  // [dst_off, dst_off + n_copy) of every arena from pristine
  size_t skip_off, skip_len;  // except [dst_off + skip_off, + skip_len) (16-byte multiples; 0: none)
  int32_t n_fill;
  uint32_t fill_byte[BATCH_INIT_FILLS];
  size_t fill_off[BATCH_INIT_FILLS], fill_len[BATCH_INIT_FILLS];
};

struct FeasArgs {
  const DevDict* dict;
  const DevCatalog* cat;
  const int64_t* vint;
  int32_t T;
  int32_t n_queries;
  int32_t mode_compatible;   // 1: Compatible(q, type, WK) (CompatibleAvailableFilter); 0: type.Intersects(q)
  int32_t pad_;              // bits kernel: bit 0 = write the cheapest-price stream with non-temporal stores
  const uint8_t* q_reqs;     // [Q] KReqs
  const int64_t* q_requests; // [Q][NRES]
  uint64_t* out_mask;        // [Q][tiles]
  double* out_cheapest;      // [Q][ch_stride] (the first T of each row) or null
  int32_t bits;              // 1: bitsets over the catalogue (feasibility_quad_kernel when T <= 1024, else
                             // feasibility_bits_kernel), 0: feasibility_kernel
  int32_t blocks;            // its grid (rows are strided over the waves)
  int32_t one_row;           // 1: feasibility_bits_kernel at any T (its cross-check, KP_FEAS_ONE_ROW)
  int32_t ch_stride;         // doubles per out_cheapest row: T rounded up to whole 128-byte lines (rows start aligned)
  uint64_t* out_classes;     // [Q] compact result: the row's compatible offering classes (kp_filter_run_compact), or null
};

// ---- launch-side selection (kp_launch_select) ------------------------------------------------------
#define LAUNCH_CAP 1024  // instance types per request on the device path
struct LaunchOut {  // kp_launch_result as the device writes it
  int32_t status, capacity_type;
  uint32_t n_types, n_overrides;
  int32_t failed_filter;
  uint32_t n_compatible, rejected_exotic, rejected_spot;
  int32_t od_fallback_warning, reservation_type;
  uint32_t rejected_reservation;
  int32_t pad_;
};
struct LaunchArgs {
  const DevDict* dict;
  const DevCatalog* cat;
  const int64_t* vint;
  int32_t n;                  // requests
  int32_t max_types;          // Truncate limit (0: none)
  int32_t spot_bit, od_bit;   // dictionary value bits of karpenter.sh/capacity-type spot / on-demand (-1: absent)
  int32_t ct_key;             // dictionary key of karpenter.sh/capacity-type
  int32_t MO;                 // offerings per type (stride of ofs_cls)
  uint64_t cls_spot, cls_od;  // offering classes whose capacity type is spot / on-demand
  int32_t res_bit, pad0_;     // dictionary value bit of karpenter.sh/capacity-type reserved (-1: absent)
  uint64_t cls_res;           // offering classes whose capacity type is reserved
  uint64_t cls_rt0, cls_rt1;  // classes whose capacity-reservation-type is default / capacity-block
  const double* price_all;    // [T][C] cheapest offering of each class, any availability (CapacityBlockFilter)
  const int32_t* rcap;        // [T][C] greatest reservation capacity over the class's available offerings
  const uint8_t* q_reqs;      // [n] KReqs
  const int64_t* q_requests;  // [n][NRES]
  const uint32_t* list_off;   // [n+1] CSR of the requests' instance-type lists
  const uint32_t* list;
  const uint64_t* exotic;     // [TW] ExoticInstanceTypeFilter's exotic types (metal size or accelerator capacity)
  const int8_t* cls_zone;     // [C] index of the class's zone in the subnet zones, -1: no subnet
  const uint8_t* ofs_cls;     // [T][MO] offering classes of each type in offering order, 0xFF: end
  uint32_t ovr_stride;        // out_overrides entries per request
  LaunchOut* out;
  uint32_t* out_types;        // [n][max_types]
  uint32_t* out_overrides;    // [n][ovr_stride]
  uint64_t* stats;            // [2]: types evaluated, algorithmic bytes
};
hipError_t launch_launch(const LaunchArgs& a, hipStream_t s);

// ---- consolidation simulations (kp_cluster_simulate) -------------------------------------------
// One in-flight NodeClaim (a simulation with a second one is a no-op, so it stops there).
struct SimNC {
  KReqs reqs;
  uint64_t X[KP_MAX_TYPE_WORDS];
  int64_t requests[KP_NRES];
  int64_t maxalloc[KP_NRES];
  int32_t fitj[KP_NRES];
  int32_t tmpl, taintset, ver, pad_;
  uint64_t hp;  // used host-port bits
};

// kp_sim_result as the device writes it (same layout as the ABI struct)
struct SimOut {
  int32_t decision;
  uint32_t nodepool;
  double candidate_price, replacement_price, savings;
  uint32_t n_options, n_pods;
};

struct SimArgs {
  const DevDict* dict;
  const DevCatalog* cats;
  int32_t n_catalogs;
  int32_t SL;                        // shape-levels
  const int64_t* vint;
  // shapes (x relaxation levels), as in SolveArgs
  const int32_t* shape_level_base;
  const int32_t* shape_nlevels;
  const int32_t* sl_shape;           // [SL] shape of a shape-level
  const uint8_t* shape_reqs;
  const uint64_t* shape_negop;
  const int64_t* shape_requests;
  const uint64_t* shape_tolerates;
  const uint64_t* shape_pvp;
  const int32_t* pvp_base;
  const int32_t* pvp_slot;
  // templates
  int32_t n_tmpl;
  const uint8_t* tmpl_reqs;
  const int32_t* tmpl_taintset;
  const int32_t* tmpl_catalog;
  const int32_t* tmpl_nodepool;
  const uint64_t* tmpl_X;
  const int64_t* tmpl_daemon;
  const uint32_t* tmpl_limit_present;  // [NT] NodePool limits: filterByRemainingResources for the new NodeClaim
  const int64_t* tmpl_remaining;       // [NT][NRES]
  // existing nodes in upstream order (initialized first, then name); position e
  int32_t E, EW;
  const uint16_t* ex_code;           // [K][E] value bit of the node's label for key k, 0xFFFF: no label
  const int32_t* ex_taintset;        // [E]
  const int64_t* ex_available;       // [E][NRES]
  const int64_t* ex_requests;        // [E][NRES]
  const uint8_t* ex_init;            // [E]
  // host ports (see SolveArgs): static used bits per node; touched nodes keep theirs in s_ovlhp
  int32_t hp_any;
  const uint64_t* shape_hp_conf;     // [S]
  const uint64_t* shape_hp_add;      // [S]
  const uint64_t* ex_hp;             // [E]
  uint64_t* s_ovlhp;                 // [slot][E] (valid where the node is touched)
  // precomputed per shape-level (sim_prep_kernel / sim_usable_kernel)
  uint64_t* usable;                  // [SL][EW] CanAdd on the snapshot: tolerated, compatible, fits
  SimNC* tres;                       // [SL] addToNewNodeClaim outcome (tmpl -1: none)
  // pods every simulation schedules besides those of S: the deleting nodes' and the pending ones
  const uint64_t* base_excl;         // [EW] deleting nodes (never destinations)
  const uint32_t* base_keys;         // [n_base] their queue ranks
  int32_t n_base;
  const uint8_t* pod_kind;           // [P] 0 on a node, 1 on a deleting node, 2 pending
  // pods (all pods of the cluster)
  const int32_t* pod_shape;          // [P]
  const uint32_t* pod_rank;          // [P] position in byCPUAndMemoryDescending order
  const uint32_t* rank_pod;          // [P]
  // cluster nodes, input order
  const int32_t* node_pos;           // [N] existing position
  const uint32_t* node_pod_off;      // [N+1]
  const uint32_t* node_pods;
  const double* node_price;          // [N] cheapest label-compatible offering of its type
  const uint8_t* node_flags;         // [N] bit0 priced, bit1 capacity-type label = spot
  const uint32_t* node_name;         // [N] type-name id
  const uint32_t* type_name;         // [n_catalogs][T] type-name id
  int32_t spot_bit, od_bit, ct_key;
  uint32_t req_res_mask;
  int32_t RU;                        // requested resources (popcount of req_res_mask)
  int8_t ru_res[KP_NRES];            // resource of overlay column u
  int32_t max_types;
  int32_t multi_node;
  int32_t spot_to_spot;              // SpotToSpotConsolidation feature gate
  int32_t wave_lds;                  // dynamic LDS bytes per wave (bitmaps + pod queue / option sort)
  // batch
  int32_t n_subsets;
  const uint32_t* sub_off;
  const uint32_t* sub_nodes;
  int32_t cap;                       // pods per simulation the LDS region holds
  int32_t cap2;                      // power of two >= max(cap, 2 * sorted types)
  // per-wave scratch (slot = global wave id)
  int32_t n_slots;
  uint64_t* s_pod;                   // [slot][cap] epoch<<40 | level<<32 | lastLen
  int32_t* s_start;                  // [slot][SL] first existing position not yet known to fail
  int64_t* s_ovl;                    // [slot][E][RU] requests of existing nodes touched by the simulation
  SimNC* s_nc;                       // [slot]
  int32_t* s_ncfail;                 // [slot][SL]
  SimOut* out;                       // [n_subsets]
  uint64_t* stats;                   // [8] attempts, bytes, pops, existing words scanned, -, cancelled
  const int32_t* cancel;             // kp_cancel flag (host-mapped) or null: polled between a wave's subsets
};

// kp_consolidate_argmin: per-block partial bests, and the record each rank contributes to the all-gather
struct ArgmaxPart {
  double savings;
  int64_t index;  // -1: no non-no-op decision in the range
  uint64_t counts[4];  // no-op, delete, replace, pod-queue overflows
};
struct CommBest {
  int64_t index;  // global subset index, -1: every decision of the rank was a no-op
  uint64_t counts[4];  // no-op, delete, replace, pod-queue overflows
  SimOut rec;
};
hipError_t launch_argmax(const SimOut* out, int n, ArgmaxPart* part, int n_parts, int64_t base, CommBest* dst,
                         hipStream_t s);

hipError_t launch_sim_prep(const SimArgs& a, hipStream_t s);
hipError_t launch_sim(const SimArgs& a, int blocks, size_t dyn_lds, hipStream_t s);
const void* sim_kernel_ptr();
#define SIM_WAVES 4

hipError_t launch_solve(const SolveArgs& a, int nw, size_t dyn_lds, hipStream_t s);
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s);
hipError_t launch_solve_batch(const SolveArgs& a0, const SolveArgs* dev_args, int n, size_t dyn_lds, hipStream_t s);
hipError_t launch_finalize_batch(const FinalizeArgs& a0, const FinalizeArgs* dev_args, int n, hipStream_t s);
hipError_t launch_batch_init(const BatchInitArgs& a, int n_arenas, hipStream_t s);
hipError_t launch_feasibility(const FeasArgs& a, hipStream_t s);

