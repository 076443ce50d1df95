// kp_kernels.hip — CDNA4 (gfx950) kernels of the Karpenter bin-packing hot path.
//
//  solve_kernel       upstream Scheduler.Solve (FFD). The whole pod loop runs device-resident in ONE
//                     workgroup per Solve; each wave evaluates one placement candidate (existing node,
//                     in-flight NodeClaim or NodeClaimTemplate) with the exact requirement algebra held one
//                     64-bit word per lane (kp_model.h), and NodeClaim.Add's instance-type filter
//                     (upstream filterInstanceTypesByRequirements) as bitmask algebra over the catalogue.
//  finalize_kernel    Results.TruncateInstanceTypes: cheapest compatible available offering per option
//                     (min over offering classes), OrderByPrice (price asc, name asc) + cut to max.
//  feasibility_kernel CompatibleAvailableFilter (R:pkg/providers/instance/filter/filter.go:39-64) for many
//                     (requirements, requests) rows × one catalogue: lane = instance type, ballot -> mask
//                     words, cheapest offering by a per-lane min over offering classes.
//
// No MFMA: the path is bitwise/integer. Wave = 64 lanes everywhere.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "kp/kp_abi.h"
#include "kp_device.h"
#include "kp_model.h"

#define LANE ((int)(threadIdx.x & 63))
// The file builds as two translation units (Makefile): KP_TU 1 = the Solve, template, finalize, launch and
// consolidation kernels with their launchers (scheduled for ILP: the single-wave Solve loop is issue-bound), KP_TU 2 =
// the filter kernels and launch_feasibility (the default scheduler: measured 2.6 % faster there). 3 = both.
#ifndef KP_TU
#define KP_TU 3
#endif
// Measurement knobs (FASTLANE, FL_NOTIME, FT_FINE, SORT_DIAG, EX_DIAG, FEASQ_SKIP_EVAL, the scan / grid shapes) are
// set only by the tools/ variant builds, which force-include tools/kp_diag.h (KP_DIAG_BUILD). Here they take their
// production values; a -D of any of them in any other build is an error, so no stray flag can turn a production
// kernel into a measurement stub.
#if !defined(KP_DIAG_BUILD) &&                                                                                       \
    (defined(FASTLANE) || defined(FL_NOTIME) || defined(FT_FINE) || defined(FAST_SCAN_MAX) ||                        \
     defined(FAST_CHK_LIVE) || defined(FAST_EX_ROUNDS) || defined(FAST_CONT) || defined(SORT_DIAG) || defined(EX_DIAG) || defined(FX_DIAG) || defined(FEAS_MAX_BLOCKS) ||                 \
     defined(FEASQ_EW) || defined(FEASQ_ROWS) || defined(FEASQ_B128) || defined(FEASQ_SKIP_EVAL) || defined(FL_SKIP) ||  \
     defined(SIM_WPE) || defined(FEASQ_MINW))
#error "a measurement knob is set outside a tools/ variant build (tools/kp_diag.h)"
#endif
#ifndef KP_DIAG_BUILD
#define KP_DIAG_BUILD 0
#endif
#ifndef FASTLANE
#define FASTLANE 1  // solve_kernel: wave-0 fast lane for merge-free placements (0 = full path only)
#endif
#ifndef FL_NOTIME
#define FL_NOTIME 1  // the fast lane's per-phase s_memtime probes are compiled out (their registers cost 3.7 % even
                     // when KP_TIMING is off); the diagnostic build (tools/build_fine.sh) turns them back on
#endif
#ifndef FT_FINE
#define FT_FINE 0  // diagnostic: finer fast-lane probes (FTF) in place of the full path's attempt split
#endif
#ifndef FAST_SCAN_MAX
#define FAST_SCAN_MAX 512  // longest first-fit scan (positions) the fast lane takes on; longer: the 4-wave pre-pass
#endif
#ifndef FAST_CHK_LIVE
#define FAST_CHK_LIVE 8  // chunked order: live (not dead) chunks the fast lane scans before the 4-wave pre-pass takes over
#endif
#ifndef FAST_EX_ROUNDS
#define FAST_EX_ROUNDS 8  // existing nodes: 64-position rounds the fast lane scans before the 4-wave pre-pass takes over
#endif
#ifndef FAST_CONT
#define FAST_CONT 1  // the continuation round (the previous pod's NodeClaim tested from registers first)
#endif
#ifndef FL_SKIP
#define FL_SKIP 0  // diagnostic cost attribution, WRONG PLACEMENTS: bit 0 no sort replay, bit 1 no mutation stack
#endif             // (cursor as stored), bit 2 no statistics counters

// Explicit address spaces: LDS data reached through a pointer would otherwise be read with FLAT loads (which wait
// on the vector-memory counter too and take the long path); global rows get global_load.
#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))
// raw buffer descriptor word 3 for gfx9-family parts (gfx950): 32-bit data format, no swizzle; with stride 0 the
// record count is in bytes and an access whose VGPR + immediate offset is at or past it returns 0 / is dropped
// (callers keep the SGPR offset 0: the range check is only relied on for the VGPR + immediate part)
#define KP_BUF_DWORD3 0x00020000
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#define FITV_RES 4      // requested resources whose Fits thresholds are staged in LDS
#define FITV_CAP 1024   // distinct allocatable values per staged resource

// ------------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------------
// wave-uniform value made provably uniform (SGPR): values read from LDS or global memory at a uniform address are
// uniform in fact, but where the compiler cannot prove it the loop and branches around them become divergent code
__device__ __forceinline__ int U(int x) { return __builtin_amdgcn_readfirstlane(x); }
// Branch-weight hints for the single-wave Solve loop: the block placement makes the hinted-likely successor the
// fall-through, and a taken branch costs a single wave ~20 cycles of instruction refetch (tools/micro/issue.hip)
#define LIKELY(x) __builtin_expect(!!(x), 1)
#define UNLIKELY(x) __builtin_expect(!!(x), 0)
// the value's load has completed here (the compiler places the wait at this point, not at a later join)
#define READY(x) asm volatile("" ::"v"(x))
__device__ __forceinline__ uint64_t U64(uint64_t x) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
// cooperative copy of a plain descriptor into LDS, one 32-bit word per thread (a single thread's copy of the
// ~2.6 KB DevDict is hundreds of serial loads: microseconds per workgroup)
template <class S>
__device__ __forceinline__ void block_copy(S& dst, const S* src) {
  static_assert(sizeof(S) % 4 == 0, "descriptor size");
  for (int i = threadIdx.x; i < (int)(sizeof(S) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t*>(&dst)[i] = reinterpret_cast<const uint32_t*>(src)[i];
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    int64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}
// broadcast lane `src` (wave-uniform) to the wave: two v_readlane, no LDS crossbar
__device__ __forceinline__ uint64_t lane_bcast(uint64_t v, int src) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, src);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int64_t lane_bcast_i64(int64_t v, int src) { return (int64_t)lane_bcast((uint64_t)v, src); }
__device__ __forceinline__ int key_word(const DevDict& D, int k, int i) { return i == 0 ? k : D.ovf[k] + i - 1; }

// Parsed integers of the value bits (vint[w*64 + b]): words w < nl from an LDS copy (the bounded keys' first
// words, staged once per kernel), the rest from global memory.
struct VInt {
  const int64_t LDS* l;
  const int64_t* g;
  int nl;
  __device__ __forceinline__ int64_t at(int w, int lane) const { return w < nl ? l[w * 64 + lane] : g[w * 64 + lane]; }
};
__device__ __forceinline__ VInt vint_global(const int64_t* g) { return VInt{nullptr, g, 0}; }

// withinIntPtrs over every word of the keys in bk, one wave-wide pass per word: lane b tests value bit b
// (coalesced 512 B read of the word's parsed integers) and a ballot forms the word's mask. Returns this lane's
// word mask (all ones when the lane's key is not in bk). Replaces a per-lane serial walk over the set bits,
// whose dependent loads made bounded-key merges the longest chain of an attempt.
__device__ __forceinline__ uint64_t bounds_mask(const DevDict& D, uint64_t bk, uint64_t hgt, uint64_t hlt,
                                                const int64_t* gt, const int64_t* lt, const VInt& vint) {
  const int lane = LANE;
  uint64_t out = ~0ull;
  while (bk) {
    const int kk = __builtin_ctzll(bk);
    bk &= bk - 1;
    const bool hg = (hgt >> kk) & 1, hl = (hlt >> kk) & 1;
    const int64_t g = gt[kk], l = lt[kk];
    uint64_t wm = 1ull << kk;
    if ((D.multiword >> kk) & 1) wm |= D.ovfmask[kk];
    while (wm) {
      const int w = __builtin_ctzll(wm);
      wm &= wm - 1;
      const int64_t x = vint.at(w, lane);
      const bool ok = ((D.vint_ok[w] >> lane) & 1) && (!hg || x > g) && (!hl || x < l);
      const uint64_t m = __ballot(ok);
      if (lane == w) out = m;
    }
  }
  return out;
}

// bounds_mask with the bound slots held by the lanes (lane k: key k's gt / lt) and the parsed integers of the staged
// words in LDS: no generic (FLAT) loads, whose waits would also cover every outstanding global load and store.
template <class DD>  // DevDict in LDS, or in the constant address space (scalar loads)
__device__ __forceinline__ uint64_t bounds_mask_lanes(const DD& D, uint64_t bk, uint64_t hgt, uint64_t hlt,
                                                      int64_t gt_lane, int64_t lt_lane, const int64_t LDS* vl, int nl,
                                                      const GLB int64_t* vg) {
  const int lane = LANE;
  uint64_t out = ~0ull;
  while (bk) {
    const int kk = __builtin_ctzll(bk);
    bk &= bk - 1;
    const bool hg = (hgt >> kk) & 1, hl = (hlt >> kk) & 1;
    const int64_t g = lane_bcast_i64(gt_lane, kk), l = lane_bcast_i64(lt_lane, kk);
    uint64_t wm = 1ull << kk;
    if ((D.multiword >> kk) & 1) wm |= D.ovfmask[kk];
    while (wm) {
      const int w = __builtin_ctzll(wm);
      wm &= wm - 1;
      int64_t x;
      if (w < nl) x = vl[w * 64 + lane];
      else x = vg[w * 64 + lane];
      const bool ok = ((D.vint_ok[w] >> lane) & 1) && (!hg || x > g) && (!hl || x < l);
      const uint64_t m = __ballot(ok);
      if (lane == w) out = m;
    }
  }
  return out;
}

// Key masks + bound slots of one requirement set; values stay in registers (one word per lane).
struct ReqView {
  uint64_t present, compl_, hgt, hlt, hmin, nz, dne;
  const int64_t* gt;
  const int64_t* lt;
  const int32_t* minv;
};

// A catalogue descriptor staged in LDS with its small tables (offering classes, Fits threshold counts), so that a
// filter step reads them with ds_read instead of a global round trip per field.
#define HDR_CLS 16
struct CatHdr {
  DevCatalog d;
  OfferClass cls[HDR_CLS];     // valid when D.C <= HDR_CLS
  int32_t fit_n[KP_NRES];
  int32_t fit_slot[KP_NRES];   // row of the kernel's LDS fit-value table holding fit_vals[r], -1: global
};
// one wave fills h from the global descriptor g (lanes copy words in parallel)
__device__ __forceinline__ void hdr_fill_wave(CatHdr LDS* h, const DevCatalog* g, int C) {
  const int lane = LANE;
  constexpr int NWD = sizeof(DevCatalog) / 8;
  if (lane < NWD) reinterpret_cast<uint64_t LDS*>(&h->d)[lane] = reinterpret_cast<const uint64_t*>(g)[lane];
  const OfferClass* gc = g->cls;
  const int32_t* gn = g->fit_n;
  constexpr int CW = sizeof(OfferClass) / 8;
  static_assert(CW * HDR_CLS <= 64, "one wave copies the class table");
  if (lane < CW * HDR_CLS && lane < CW * C)
    reinterpret_cast<uint64_t LDS*>(h->cls)[lane] = reinterpret_cast<const uint64_t*>(gc)[lane];
  if (lane < KP_NRES) {
    h->fit_n[lane] = gn[lane];
    h->fit_slot[lane] = -1;
  }
}

// operator in {NotIn, DoesNotExist}: complement with values, or no complement and no values.
__device__ __forceinline__ uint64_t negop_mask(uint64_t present, uint64_t compl_, uint64_t nz) {
  return present & ((compl_ & nz) | (~compl_ & ~nz));
}

// keys with at least one value bit: word k is key k's first word, so one ballot + the few overflow keys
template <class DD>
__device__ __forceinline__ uint64_t nz_keys(const DD& D, uint64_t v) {
  const uint64_t bal = __ballot(v != 0 && LANE < D.W);
  uint64_t nz = bal & D.firstmask;
  const uint64_t ov = bal & ~D.firstmask;
  if (ov) {
    uint64_t mk = D.multiword;
    while (mk) {
      const int k = __builtin_ctzll(mk);
      mk &= mk - 1;
      if (ov & D.ovfmask[k]) nz |= 1ull << k;
    }
  }
  return nz;
}

// Per-wave LDS scratch holding a merged requirement set's bound slots.
struct WaveSlots {
  int64_t gt[KP_MAX_BOUND_KEYS];
  int64_t lt[KP_MAX_BOUND_KEYS];
  int32_t minv[KP_MAX_BOUND_KEYS];
};

// A candidate's requirement set as registers: key masks (wave-uniform) + this lane's value word and bound slot.
// Loading it is one batch of independent loads, issued before anything that depends on it.
struct CandReq {
  uint64_t P, C, hgt, hlt, hmin, v;
  int64_t gt, lt;
  int32_t minv;
};
__device__ __forceinline__ CandReq load_cand(const DevDict& D, const KReqs* A) {
  const int lane = LANE;
  CandReq c;
  c.P = A->present;
  c.C = A->compl_;
  c.hgt = A->hgt;
  c.hlt = A->hlt;
  c.hmin = A->hmin;
  c.v = lane < D.W ? A->vals[lane] : 0;
  const bool b = lane < D.KB;
  c.gt = b ? A->gt[lane] : 0;
  c.lt = b ? A->lt[lane] : 0;
  c.minv = b ? A->minv[lane] : 0;
  return c;
}

// Requirements.Compatible(A, B, allowUndefined) followed by A.Add(B) (= per key Requirement.Intersection).
// On success: m_v = merged value word of this lane, rv = merged key masks, slots = merged bounds.
__device__ __forceinline__ bool merge_compatible(const DevDict& D, const CandReq& A, const KReqs* B, uint64_t b_negop, bool allow_wk,
                                 uint64_t& m_v, ReqView& rv, WaveSlots* slots, const VInt& vint) {
  const int lane = LANE;
  const int k = lane < D.W ? (int)D.wkey[lane] : -1;
  const uint64_t aP = A.P, bP = B->present;
  const uint64_t shared = aP & bP;
  // (a) keys the pod defines but the candidate does not: only NotIn/DoesNotExist (or well-known) pass
  uint64_t undef = bP & ~aP & ~b_negop;
  if (allow_wk) undef &= ~D.wellknown;
  if (undef) return false;
  const uint64_t a_v = A.v;
  const uint64_t b_v = lane < D.W ? B->vals[lane] : 0;
  const uint64_t aC = A.C & aP, bC = B->compl_ & bP;
  // bound slots: lane l < KB owns key l
  bool hg = false, hl = false, dneb = false;
  if (lane < D.KB) {
    const bool inA = (aP >> lane) & 1, inB = (bP >> lane) & 1;
    const bool agt = inA && ((A.hgt >> lane) & 1), bgt = inB && ((B->hgt >> lane) & 1);
    const bool alt = inA && ((A.hlt >> lane) & 1), blt = inB && ((B->hlt >> lane) & 1);
    hg = agt || bgt;
    hl = alt || blt;
    const int64_t g = agt && bgt ? max(A.gt, B->gt[lane]) : (agt ? A.gt : (bgt ? B->gt[lane] : 0));
    const int64_t l = alt && blt ? min(A.lt, B->lt[lane]) : (alt ? A.lt : (blt ? B->lt[lane] : 0));
    const bool amin = inA && ((A.hmin >> lane) & 1), bmin = inB && ((B->hmin >> lane) & 1);
    const int32_t mv = amin && bmin ? max(A.minv, B->minv[lane]) : (amin ? A.minv : (bmin ? B->minv[lane] : 0));
    dneb = inA && inB && hg && hl && g >= l;
    slots->gt[lane] = g;
    slots->lt[lane] = l;
    slots->minv[lane] = mv;
  }
  const uint64_t hgt_any = __ballot(hg), hlt_any = __ballot(hl), dne = __ballot(dneb);
  wave_sync();
  uint64_t v = 0;
  if (k >= 0) {
    if ((shared >> k) & 1) {
      const bool c1 = (aC >> k) & 1, c2 = (bC >> k) & 1;
      v = (c1 && c2) ? (a_v | b_v) : c1 ? (b_v & ~a_v) : c2 ? (a_v & ~b_v) : (a_v & b_v);
      if ((dne >> k) & 1) v = 0;  // gt >= lt: NewRequirementWithFlexibility(key, DoesNotExist, minValues)
    } else {
      v = ((aP >> k) & 1) ? a_v : b_v;
    }
  }
  const uint64_t bk = (hgt_any | hlt_any) & shared & ~dne;
  if (bk) v &= bounds_mask(D, bk, hgt_any, hlt_any, slots->gt, slots->lt, vint);
  m_v = v;
  const uint64_t compl_new = ((aC & bC) | (aC & ~bP) | (bC & ~aP)) & ~dne;
  const uint64_t nz = nz_keys(D, v);
  rv.present = aP | bP;
  rv.compl_ = compl_new;
  rv.hgt = hgt_any & compl_new;
  rv.hlt = hlt_any & compl_new;
  rv.hmin = (A.hmin & aP) | (B->hmin & bP);
  rv.nz = nz;
  rv.dne = dne;
  rv.gt = slots->gt;
  rv.lt = slots->lt;
  rv.minv = slots->minv;
  // (b) Intersects over shared keys: empty intersection is an error unless both ops are NotIn/DNE
  const uint64_t empty = shared & (dne | (~compl_new & ~nz));
  const uint64_t nzA = nz_keys(D, a_v);
  const uint64_t negA = negop_mask(aP, aC, nzA);
  return (empty & ~(negA & b_negop)) == 0;
}
__device__ __forceinline__ bool merge_compatible(const DevDict& D, const KReqs* A, const KReqs* B, uint64_t b_negop,
                                                 bool allow_wk, uint64_t& m_v, ReqView& rv, WaveSlots* slots,
                                                 const VInt& vint) {
  return merge_compatible(D, load_cand(D, A), B, b_negop, allow_wk, m_v, rv, slots, vint);
}

// Allowed-value bits (Requirement.Has) of this lane's word under requirement set rv; absent key -> all.
__device__ __forceinline__ uint64_t allowed_word(const DevDict& D, const ReqView& rv, uint64_t v, const VInt& vint) {
  const int lane = LANE;
  const uint64_t bk = (rv.hgt | rv.hlt) & rv.present & rv.compl_ & ((1ull << D.KB) - 1);
  const uint64_t bm = bk ? bounds_mask(D, bk, rv.hgt, rv.hlt, rv.gt, rv.lt, vint) : ~0ull;
  if (lane >= D.W) return 0;
  const int k = D.wkey[lane];
  if (!((rv.present >> k) & 1)) return D.validbits[lane];
  if ((rv.compl_ >> k) & 1) return ~v & D.validbits[lane] & bm;
  return v;
}

__device__ __forceinline__ bool bit_of(uint64_t allowed_lane_word, int bit) {
  const uint64_t w = lane_bcast(allowed_lane_word, bit >> 6);
  return (w >> (bit & 63)) & 1;
}

// Offering classes compatible with requirement set rv (Offerings.Compatible): a reservation key the class does not
// carry is DoesNotExist, compatible when rv leaves the key out or admits its absence.
// RES = false (Solve, consolidation: their catalogues hold no reservation classes) skips the reservation bits.
template <bool RES = false, class ClsP, class DD>
__device__ uint64_t allowed_classes(const DD& D, ClsP cls_tab, const ReqView& rv, uint64_t allowed, uint64_t negR) {
  if (!RES && D.res_any) return allowed_classes<true>(D, cls_tab, rv, allowed, negR);  // Solve over reservations
  const bool res_ok = !(rv.present & D.resid_key_bit) || (negR & D.resid_key_bit);
  const bool rt_ok = !(rv.present & D.restype_key_bit) || (negR & D.restype_key_bit);
  // lane c evaluates class c: its value bits are fetched from the owning lanes' allowed words
  const int lane = LANE;
  int ct_bit = 0, zone_bit = -1, zid_bit = -1, rid_bit = -1, rt_bit = -1;
  if (lane < D.C) {
    ct_bit = cls_tab[lane].ct_bit;
    zone_bit = cls_tab[lane].zone_bit;
    zid_bit = cls_tab[lane].zid_bit;
    if (RES) {
      rid_bit = cls_tab[lane].rid_bit;
      rt_bit = cls_tab[lane].rt_bit;
    }
  }
  const uint64_t w1 = __shfl(allowed, ct_bit >> 6, 64);
  const uint64_t w2 = __shfl(allowed, zone_bit >= 0 ? zone_bit >> 6 : 0, 64);
  const uint64_t w3 = __shfl(allowed, zid_bit >= 0 ? zid_bit >> 6 : 0, 64);
  bool ok = lane < D.C && ((w1 >> (ct_bit & 63)) & 1) && (zone_bit < 0 || ((w2 >> (zone_bit & 63)) & 1)) &&
            (zid_bit < 0 || ((w3 >> (zid_bit & 63)) & 1));
  if (RES && __ballot(rid_bit >= 0 || rt_bit >= 0)) {  // reservation classes (launch / filter plans only)
    const uint64_t w4 = __shfl(allowed, rid_bit >= 0 ? rid_bit >> 6 : 0, 64);
    const uint64_t w5 = __shfl(allowed, rt_bit >= 0 ? rt_bit >> 6 : 0, 64);
    ok = ok && (rid_bit < 0 ? res_ok : ((w4 >> (rid_bit & 63)) & 1)) && (rt_bit < 0 ? rt_ok : ((w5 >> (rt_bit & 63)) & 1));
  } else {
    ok = ok && res_ok && rt_ok;
  }
  return __ballot(ok);
}

// first j in [0, n) with vals[j] >= q (ascending vals), n if none; 64-ary search across the wave.
template <class ValP>
__device__ int wave_lower_bound(ValP vals, int n, int64_t q, uint64_t* bytes) {
  const int lane = LANE;
  int lo = 0, hi = n;  // vals[j] < q for j < lo; answer <= hi
  while (lo < hi) {
    const int span = hi - lo;
    if (span <= 64) {
      const bool ge = lane < span && vals[lo + lane] >= q;
      const uint64_t bal = __ballot(ge);
      *bytes += 8ull * span;
      return bal ? lo + __builtin_ctzll(bal) : hi;
    }
    const int step = (span + 63) / 64;
    const int idx = lo + lane * step;
    const bool ge = idx < hi && vals[idx] >= q;
    const uint64_t bal = __ballot(ge);
    *bytes += 512;
    if (!bal) {
      lo = lo + min(63, (hi - 1 - lo) / step) * step + 1;  // past the last sample taken (< hi)
    } else {
      const int f = __builtin_ctzll(bal);
      if (f == 0) return lo;
      const int nlo = lo + (f - 1) * step + 1;
      hi = lo + f * step;
      lo = nlo;
    }
  }
  return lo;
}

// minValues over a type set (SatisfiesMinValues): for every key in `mk`, the remaining types (X: this lane's
// word) must carry at least minv[k] distinct values of it.
__device__ bool minvalues_ok(const DevDict& D, const uint16_t* code_tab, const uint64_t* TM, uint64_t mk, const int32_t* minv, uint64_t X,
                             uint32_t* scratch) {
  const int lane = LANE;
  const int TW = D.TW;
  bool ok = true;
  while (mk) {
    const int k = __builtin_ctzll(mk);
    mk &= mk - 1;
    const int nw = (D.nval[k] + 63) >> 6;
    int count = 0;
    if ((D.single_valued >> k) & 1) {
      for (int w = lane; w < 2 * nw; w += 64) scratch[w] = 0;
      wave_sync();
      uint64_t m = lane < TW ? X : 0;
      while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        const uint16_t code = code_tab[(size_t)k * D.T + lane * 64 + b];
        if (code < 0xFFFD) {
          const int cw = code >> 6;
          const int rel = (cw == k ? 0 : (cw - D.ovf[k] + 1) * 64) + (code & 63);  // ordinal within key k
          atomicOr(&scratch[rel >> 5], 1u << (rel & 31));
        }
      }
      wave_sync();
      int c = 0;
      for (int w = lane; w < 2 * nw; w += 64) c += __builtin_popcount(scratch[w]);
      count = wave_sum(c);
      wave_sync();
    } else {
      for (int wi = 0; wi < nw; wi++) {
        const int w = key_word(D, k, wi);
        uint64_t vb = D.validbits[w];
        while (vb) {
          const int b = __builtin_ctzll(vb);
          vb &= vb - 1;
          const uint64_t hit = lane < TW ? (X & TM[(size_t)(w * 64 + b) * TW + lane]) : 0;
          count += __ballot(hit != 0) ? 1 : 0;
        }
      }
    }
    if (count < minv[k]) ok = false;
  }
  return ok;
}

// Row list: the type-mask rows one filter step ANDs into X, grouped (a group's rows are ORed, then ANDed into X).
// Building it needs no global memory (LDS + scalar work), so all of its loads go out together in one batch
// instead of one dependent round trip per key / resource / offering class. Per-wave LDS: RL_CAP row pointers.
#define RL_CAP 16
typedef const uint64_t GLB* RowPtr;
struct RowBatch {
  RowPtr LDS* rows;       // per-wave LDS
  int n;
  uint32_t endm;          // bit i: row i closes a group
  uint64_t acc;
};
// Rows are loaded four at a time (one batch of independent loads per group): a step with few rows (the usual
// 3-6) executes one group instead of a fully unrolled RL_CAP-slot body.
__device__ __forceinline__ void rl_flush(RowBatch& L, uint64_t& X, int TW) {
  if (L.n == 0) return;
  wave_sync();
  const int lane = LANE;
  const bool lv = lane < TW;
  for (int g = 0; g < L.n; g += 4) {
    const int m = L.n - g;
    const uint64_t w0 = lv ? L.rows[g][lane] : 0;
    const uint64_t w1 = (m > 1 && lv) ? L.rows[g + 1][lane] : 0;
    const uint64_t w2 = (m > 2 && lv) ? L.rows[g + 2][lane] : 0;
    const uint64_t w3 = (m > 3 && lv) ? L.rows[g + 3][lane] : 0;
    const uint32_t e = L.endm >> g;
    L.acc |= w0;
    if (e & 1) X &= L.acc, L.acc = 0;
    if (m > 1) {
      L.acc |= w1;
      if (e & 2) X &= L.acc, L.acc = 0;
    }
    if (m > 2) {
      L.acc |= w2;
      if (e & 4) X &= L.acc, L.acc = 0;
    }
    if (m > 3) {
      L.acc |= w3;
      if (e & 8) X &= L.acc, L.acc = 0;
    }
  }
  L.n = 0;
  L.endm = 0;
  wave_sync();
}
// overflow path (more than RL_CAP rows in one step): a plain loop, kept small so that the push sites stay compact
__device__ __forceinline__ void rl_flush_slow(RowBatch& L, uint64_t& X, int TW) {
  wave_sync();
  const int lane = LANE;
#pragma unroll 1
  for (int i = 0; i < L.n; i++) {
    const uint64_t w = lane < TW ? L.rows[i][lane] : 0;
    L.acc |= w;
    if ((L.endm >> i) & 1) {
      X &= L.acc;
      L.acc = 0;
    }
  }
  L.n = 0;
  L.endm = 0;
  wave_sync();
}
__device__ __forceinline__ void rl_push(RowBatch& L, uint64_t& X, int TW, const uint64_t* row, bool end) {
  if (L.n == RL_CAP) rl_flush_slow(L, X, TW);
  if (LANE == 0) L.rows[L.n] = (RowPtr)row;
  if (end) L.endm |= 1u << L.n;
  L.n++;
}

// resources.Fits(total, allocatable) as row pushes: per requested resource a threshold mask. A NodeClaim's
// totals only grow, so the threshold index does too: probe 64 entries past the cached index first. Returns the
// threshold indices (lane r: resource r); `zero` is set when some resource fits no type.
__device__ __forceinline__ int32_t fits_rows(const DevDict& D, const CatHdr LDS* H, RowBatch& L, uint64_t& X,
                                             int64_t q_lane, int32_t j0_lane, const int64_t LDS* fitv_lds,
                                             uint32_t rmask, uint64_t& nb, bool& zero) {
  const int lane = LANE;
  const int TW = D.TW;
  // 2) resources.Fits(total, allocatable): per requested resource, a threshold mask. A NodeClaim's totals
  //    only grow, so the threshold index does too: probe 64 entries past the cached index first.
  int32_t j_lane = 0;
  uint32_t rm = rmask;
  while (rm) {
    const int r = __builtin_ctz(rm);
    rm &= rm - 1;
    const int64_t q = lane_bcast_i64(q_lane, r);
    if (q <= 0) continue;
    const int j0 = __builtin_amdgcn_readlane(j0_lane, r);
    const int n = H->fit_n[r];
    const int slot = H->fit_slot[r];
    const int idx = j0 + lane;
    uint64_t bal;
    if (slot >= 0) {  // (unconditional reads at a clamped index, masked after)
      const int64_t fv = fitv_lds[slot * FITV_CAP + min(idx, FITV_CAP - 1)];
      bal = __ballot(idx < n && fv >= q);
    } else {
      const int64_t fv = H->d.fit_vals[(size_t)r * D.T + min(idx, D.T - 1)];
      bal = __ballot(idx < n && fv >= q);
    }
    nb += 512;
    int j;
    if (bal) j = j0 + __builtin_ctzll(bal);
    else if (j0 + 64 >= n) j = n;
    else if (slot >= 0) j = wave_lower_bound(fitv_lds + slot * FITV_CAP + j0 + 64, n - j0 - 64, q, &nb) + j0 + 64;
    else j = wave_lower_bound(H->d.fit_vals + (size_t)r * D.T + j0 + 64, n - j0 - 64, q, &nb) + j0 + 64;
    if (j >= n) zero = true;
    else rl_push(L, X, TW, H->d.fit_mask + ((size_t)r * D.T + j) * TW, true);
    nb += (uint64_t)TW * 8;
    if (lane == r) j_lane = j;
  }
  return j_lane;
}

// NodeClaim.Add's instance-type filter after a successful merge. X: this lane's word of the candidate's
// remaining types (invariant: X already passes every key the pod did not touch). q_lane: lane r < NRES holds the
// merged requests (candidate + pod) of resource r, j0_lane the candidate's cached threshold index. Returns the
// new word; jout[r] receives the threshold index of resource r.
__device__ __forceinline__ uint64_t filter_types(const DevDict& D, const CatHdr LDS* H, const ReqView& rv, uint64_t m_v,
                                                 uint64_t X, uint64_t pod_keys, const uint64_t* pvp,
                                                 const int32_t* pvp_slot, int64_t q_lane, int32_t j0_lane,
                                                 const int64_t LDS* fitv_lds, uint32_t rmask, const VInt& vint,
                                                 uint32_t* scratch, RowPtr LDS* rl, uint64_t* bytes, int32_t* jout,
                                                 uint64_t generic_keys = 0, uint64_t* tsub = nullptr,
                                                 bool min_check = true) {
  const int lane = LANE;
  const int TW = D.TW;
  uint64_t tl = tsub ? __builtin_amdgcn_s_memtime() : 0;
#define TSUB(i)                                        \
  if (tsub) {                                          \
    const uint64_t tn = __builtin_amdgcn_s_memtime(); \
    if (lane == 0) tsub[i] += tn - tl;                 \
    tl = tn;                                           \
  }
  const uint64_t negM = negop_mask(rv.present, rv.compl_, rv.nz);
  const uint64_t allowed = allowed_word(D, rv, m_v, vint);
  uint64_t nb = 0;
  bool zero = false;
  RowBatch L{rl, 0, 0, 0};
  // 1) Intersects(type, merged) for the keys the pod changed
  uint64_t keys = pod_keys & D.catalog_keys;
  while (keys) {
    const int k = __builtin_ctzll(keys);
    keys &= keys - 1;
    const bool ng = (negM >> k) & 1;
    if (((D.single_valued & ~generic_keys) >> k) & 1) {
      // X ⊆ Pass(candidate_k) and Has_merged = Has_candidate ∧ Has_pod, so for single-valued keys
      // X ∩ ∪_{Has_merged(v)} TM[v] = X ∩ ∪_{Has_pod(v)} TM[v] (precomputed PVP row, incl. NOKEY)
      rl_push(L, X, TW, pvp + (size_t)pvp_slot[k] * TW, !ng);
      if (ng) rl_push(L, X, TW, H->d.DNE + (size_t)k * TW, true);
      nb += (uint64_t)TW * 8 * (ng ? 2 : 1);
    } else {  // multi-valued keys, and keys narrowed by topology (Has_merged is no longer Has_pod there)
      rl_push(L, X, TW, H->d.NOKEY + (size_t)k * TW, false);
      if (ng) rl_push(L, X, TW, H->d.DNE + (size_t)k * TW, false);
      const int nw = (D.nval[k] + 63) >> 6;
      for (int wi = 0; wi < nw; wi++) {
        const int w = key_word(D, k, wi);
        uint64_t a = lane_bcast(allowed, w);
        while (a) {
          const int b = __builtin_ctzll(a);
          a &= a - 1;
          rl_push(L, X, TW, H->d.TM + (size_t)(w * 64 + b) * TW, false);
          nb += (uint64_t)TW * 8;
        }
      }
      L.endm |= 1u << (L.n - 1);  // close the key's group (its last row)
    }
  }
  TSUB(1);
  // 2) resources.Fits(total, allocatable)
  const int32_t j_lane = fits_rows(D, H, L, X, q_lane, j0_lane, fitv_lds, rmask, nb, zero);
  if (lane < KP_NRES) jout[lane] = j_lane;
  TSUB(2);
  // 3) some available offering compatible with the merged requirements. X already satisfies the
  //    candidate's offering keys; only a pod that constrains one of them can change the answer.
  if (pod_keys & D.offer_keys) {
    const uint64_t cls = D.C <= HDR_CLS ? allowed_classes(D, H->cls, rv, allowed, negM)
                                        : allowed_classes(D, H->d.cls, rv, allowed, negM);
    if (!cls) zero = true;
    uint64_t m = cls;
    while (m) {
      const int c = __builtin_ctzll(m);
      m &= m - 1;
      rl_push(L, X, TW, H->d.offer_avail + (size_t)c * TW, m == 0);
    }
    nb += (uint64_t)__builtin_popcountll(cls) * TW * 8;
  }
  rl_flush(L, X, TW);
  if (zero) X = 0;
  TSUB(3);
  // 4) minValues (relaxMinValues = false): distinct values of each minValues key over remaining types
  if (min_check && (rv.hmin & rv.present))
    if (!minvalues_ok(D, H->d.code, H->d.TM, rv.hmin & rv.present, rv.minv, X, scratch)) X = 0;
  TSUB(4);
#undef TSUB
  *bytes += nb;
  return X;
}

// NodeClaim.reserveOfferings (upstream nodeclaim.go; design R:designs/odcr.md:248-256) on a wave: M = the reserved
// classes (one per reservation id) compatible with the NodeClaim's new requirements (rv, m_v) that offer an available
// offering among its remaining types X; the held set becomes (held ∩ M) ∪ {c ∈ M \ held : capacity left}. Strict mode
// (ReservedOfferingModeStrict) fails when that is empty while M or held is not: returns ~0 then.
__device__ uint64_t reserve_classes(const DevDict& D, const CatHdr LDS* H, const ReqView& rv, uint64_t m_v, uint64_t X,
                                    uint64_t res_cls, uint64_t held, const int32_t LDS* cap, bool strict, const VInt& vint) {
  const int lane = LANE;
  const uint64_t negM = negop_mask(rv.present, rv.compl_, rv.nz);
  const uint64_t allowed = allowed_word(D, rv, m_v, vint);
  uint64_t cls = (D.C <= HDR_CLS ? allowed_classes<true>(D, H->cls, rv, allowed, negM)
                                 : allowed_classes<true>(D, H->d.cls, rv, allowed, negM)) & res_cls;
  uint64_t M = 0;
  while (cls) {
    const int c = __builtin_ctzll(cls);
    cls &= cls - 1;
    const uint64_t row = lane < D.TW ? H->d.offer_avail[(size_t)c * D.TW + lane] : 0;
    if (__ballot((row & X) != 0)) M |= 1ull << c;
  }
  const uint64_t free = __ballot(lane < D.C && cap[lane] > 0);
  const uint64_t nh = (held & M) | (M & ~held & free);
  return strict && !nh && (M | held) ? ~0ull : nh;
}

// A reservation commit on the wave: capacity of the newly held classes down, of the released ones up.
__device__ __forceinline__ void reserve_commit(int32_t LDS* cap, uint64_t held, uint64_t nh) {
  const int lane = LANE;
  if (lane < 64) {
    if (((nh & ~held) >> lane) & 1) cap[lane] -= 1;
    if (((held & ~nh) >> lane) & 1) cap[lane] += 1;
  }
}

// Algorithmic-byte accounting of fits_lean: bytes directly (uint64_t), or event counts the caller converts once
// (NbUnits: 512-byte threshold probes, TW-word mask rows, lower-bound bytes / 8), which keeps the hot loop's
// registers free of 64-bit accumulators.
struct NbUnits {
  uint32_t probes, rows, lb8;
};
__device__ __forceinline__ void nb_probe(uint64_t& nb, uint32_t n, int) { nb += 512ull * n; }
__device__ __forceinline__ void nb_probe(NbUnits& nb, uint32_t n, int) { nb.probes += n; }
__device__ __forceinline__ void nb_row(uint64_t& nb, uint32_t n, int TW) { nb += (uint64_t)TW * 8 * n; }
__device__ __forceinline__ void nb_row(NbUnits& nb, uint32_t n, int) { nb.rows += n; }
__device__ __forceinline__ void nb_lb(uint64_t& nb, uint64_t b) { nb += b; }
__device__ __forceinline__ void nb_lb(NbUnits& nb, uint64_t b) { nb.lb8 += (uint32_t)(b >> 3); }

// fits_filter for at most 4 requested resources (the fast lane): the threshold probes, then the (up to 4) mask
// rows as one batch of independent loads, ANDed into X. Same result and threshold indices as fits_filter.
template <class NB>
__device__ __forceinline__ uint64_t fits_lean(const DevDict& D, const CatHdr LDS* H, uint64_t X, int64_t q_lane,
                                              int32_t j0_lane, const int64_t LDS* fitv_lds, uint32_t rr, int nr,
                                              NB& nb, int32_t LDS* jout) {
  const int lane = LANE;
  const int TW = D.TW;
  // threshold indices unchanged for every requested resource (q_r <= fit_vals_r[j0_r], one LDS probe per lane):
  // X already lies in those rows (it was ANDed with them when j0 was stored), so X is the answer without loads
  {
    bool same = true;
    bool in_rr = false;
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (k < nr && (int)((rr >> (8 * k)) & 0xff) == lane) in_rr = true;
    {  // unconditional LDS reads at clamped indices, the lanes outside the requested resources masked after
      const int ln = min(lane, KP_NRES - 1);
      const int n = H->fit_n[ln];
      const int slot = H->fit_slot[ln];
      const int64_t fv = fitv_lds[max(slot, 0) * FITV_CAP + min(max(j0_lane, 0), FITV_CAP - 1)];
      same = !(in_rr && q_lane > 0) || (j0_lane < n && slot >= 0 && fv >= q_lane);
    }
    const uint64_t act = __ballot(in_rr && q_lane > 0);
    if (LIKELY(__ballot(!same) == 0)) {
      nb_probe(nb, (uint32_t)__popcll(act), TW);  // the algorithm's probe + row bytes, as below
      nb_row(nb, (uint32_t)__popcll(act), TW);
      if (lane < KP_NRES) jout[lane] = j0_lane;
      return X;
    }
  }
  const uint64_t GLB* rowp[4] = {nullptr, nullptr, nullptr, nullptr};
  bool zero = false;
  int32_t j_lane = j0_lane;  // (resources outside rr keep their index)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k >= nr) break;
    const int r = (rr >> (8 * k)) & 0xff;
    const int64_t q = lane_bcast_i64(q_lane, r);
    if (q <= 0) continue;
    const int j0 = __builtin_amdgcn_readlane(j0_lane, r);
    const int n = H->fit_n[r];
    const int slot = H->fit_slot[r];
    const int idx = j0 + lane;
    uint64_t bal;
    if (slot >= 0) {  // (unconditional reads at a clamped index, masked after)
      const int64_t fv = fitv_lds[slot * FITV_CAP + min(idx, FITV_CAP - 1)];
      bal = __ballot(idx < n && fv >= q);
    } else {
      const int64_t fv = H->d.fit_vals[(size_t)r * D.T + min(idx, D.T - 1)];
      bal = __ballot(idx < n && fv >= q);
    }
    nb_probe(nb, 1, TW);
    int j;
    if (bal) j = j0 + __builtin_ctzll(bal);
    else if (j0 + 64 >= n) j = n;
    else {
      uint64_t lb = 0;
      if (slot >= 0) j = wave_lower_bound(fitv_lds + slot * FITV_CAP + j0 + 64, n - j0 - 64, q, &lb) + j0 + 64;
      else j = wave_lower_bound(H->d.fit_vals + (size_t)r * D.T + j0 + 64, n - j0 - 64, q, &lb) + j0 + 64;
      nb_lb(nb, lb);
    }
    if (j >= n) zero = true;
    else rowp[k] = (const uint64_t GLB*)(H->d.fit_mask + ((size_t)r * D.T + j) * TW);
    nb_row(nb, 1, TW);
    if (lane == r) j_lane = j;
  }
  if (lane < KP_NRES) jout[lane] = j_lane;
  if (zero) return 0;
  const bool lv = lane < TW;
  const int lw = min(lane, TW - 1);  // (unconditional row reads at a clamped word, masked after)
  const uint64_t r0 = rowp[0] ? rowp[0][lw] : ~0ull, r1 = rowp[1] ? rowp[1][lw] : ~0ull;
  const uint64_t r2 = rowp[2] ? rowp[2][lw] : ~0ull, r3 = rowp[3] ? rowp[3][lw] : ~0ull;
  const uint64_t w0 = lv ? r0 : ~0ull, w1 = lv ? r1 : ~0ull, w2 = lv ? r2 : ~0ull, w3 = lv ? r3 : ~0ull;
  return X & w0 & w1 & w2 & w3;
}

// NodeClaim.Add when the pod's shape-level was already merged into the NodeClaim: Requirement.Intersection is
// idempotent (set ops, max/min bounds and minValues), so the merged requirements equal the NodeClaim's and its
// remaining types pass every compatibility and offering test already; only Fits over the grown totals changes
// (callers exclude topology-owning shape-levels and NodeClaims with minValues).
__device__ __forceinline__ uint64_t fits_filter(const DevDict& D, const CatHdr LDS* H, uint64_t X, int64_t q_lane,
                                                int32_t j0_lane, const int64_t LDS* fitv_lds, uint32_t rmask,
                                                RowPtr LDS* rl, uint64_t* bytes, int32_t* jout) {
  const int lane = LANE;
  uint64_t nb = 0;
  bool zero = false;
  RowBatch L{rl, 0, 0, 0};
  const int32_t j_lane = fits_rows(D, H, L, X, q_lane, j0_lane, fitv_lds, rmask, nb, zero);
  if (lane < KP_NRES) jout[lane] = j_lane;
  rl_flush(L, X, D.TW);
  if (zero) X = 0;
  *bytes += nb;
  return X;
}

// ------------------------------------------------------------------------------------------------
// Go sort.Slice (pdqsort_func) over the in-flight NodeClaims by len(Pods), executed by one lane.
// ------------------------------------------------------------------------------------------------
// P: int32_t LDS* (sort arrays in LDS) or int32_t GLB* (spilled to global memory); typed pointers keep the
// accesses ds_* / global_* instead of FLAT (which waits on both counters and takes the long path for LDS).
typedef int32_t LDS* LdsI32;
typedef int32_t GLB* GlbI32;
template <class P>
struct NCSortT {
  P ord;  // newNodeClaims (NodeClaim ids)
  P key;  // len(Pods) per NodeClaim id
  __device__ bool Less(int i, int j) const { return key[ord[i]] < key[ord[j]]; }
  __device__ void Swap(int i, int j) const {
    const int32_t t = ord[i];
    ord[i] = ord[j];
    ord[j] = t;
  }
};
struct NCSort {
  int32_t* ord;        // newNodeClaims (NodeClaim ids)
  const int32_t* key;  // len(Pods) per NodeClaim id
  __device__ bool Less(int i, int j) const { return key[ord[i]] < key[ord[j]]; }
  __device__ void Swap(int i, int j) const {
    const int32_t t = ord[i];
    ord[i] = ord[j];
    ord[j] = t;
  }
};
#include "kp_pdqsort.h"

// ------------------------------------------------------------------------------------------------
// topology spread (upstream Topology.AddRequirements / TopologyGroup.nextDomainTopologySpread / Record)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// Per-pod staging of one owned group: s_tg = {group, self, key, hostname row, maxSkew, key slot}. For a
// dictionary key, acc = registered domains d with count(d) + self - min <= maxSkew, where min is
// domainMinCount over the registered domains podDomains admits (minDomains -> 0); the counts go to LDS.
struct TopoOwn {
  int32_t g, self, key, row, maxskew, slot;
};

// AddRequirements + Compatible + Add for the owned dictionary-key groups on the merged requirements of one
// candidate (one wave): each group picks, among its acceptable domains that the candidate's requirements
// admit (nodeDomains; Exists when the key is absent), the one with the lowest count, ties to the lowest
// value ordinal (= byte order, the written spec for upstream's map-order tie); the key narrows to In{d}.
__device__ bool topo_narrow(const DevDict& D, int n, const TopoOwn* own, const uint64_t* acc, const int32_t (*cnt)[64],
                            bool allow_wk, uint64_t& m_v, ReqView& rv, const VInt& vint) {
  const int lane = LANE;
  const uint64_t allowed = allowed_word(D, rv, m_v, vint);
  uint64_t narrowed = 0, nv = m_v;
  for (int j = 0; j < n; j++) {
    const int k = own[j].key;
    if (k < 0) continue;  // hostname: checked exactly by the pre-pass (a fresh node always passes)
    const uint64_t kb = 1ull << k;
    const bool present = (rv.present & kb) != 0;
    if (!present && !(allow_wk && (D.wellknown & kb))) return false;  // topology key undefined on the node
    const uint64_t aN = present ? lane_bcast(allowed, k) : D.validbits[k];
    const uint64_t cand = acc[j] & aN;
    if (!cand) return false;
    uint64_t pick;
    if (own[j].maxskew > 0) {  // spread: the lowest count, ties to the lowest ordinal
      const bool in = (cand >> lane) & 1;
      const int c = in ? cnt[j][lane] : INT32_MAX;
      const int mc = wave_min_i32(c);
      pick = 1ull << __builtin_ctzll(__ballot(in && c == mc));
    } else if (own[j].maxskew < 0 && own[j].self) {  // pod-affinity bootstrap: the first domain the node admits
      pick = cand & (0 - cand);
    } else {  // pod (anti-)affinity: every acceptable domain (requirements.Add intersects)
      pick = cand;
    }
    if (narrowed & kb) {  // groups on one key intersect (empty: Compatible fails)
      const uint64_t both = lane_bcast(nv, k) & pick;
      if (!both) return false;
      if (lane == k) nv = both;
    } else if (lane == k) {
      nv = pick;
    }
    narrowed |= kb;
  }
  m_v = nv;
  rv.present |= narrowed;
  rv.compl_ &= ~narrowed;
  rv.hgt &= ~narrowed;
  rv.hlt &= ~narrowed;
  rv.nz |= narrowed;
  rv.dne &= ~narrowed;
  return true;
}

// ------------------------------------------------------------------------------------------------
// solve_kernel: one workgroup runs one Solve.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ const KReqs* kreq_at(const uint8_t* base, size_t i) {
  return reinterpret_cast<const KReqs*>(base + i * sizeof(KReqs));
}

// An existing node's requirements to read: a batched simulation's own copy once it wrote one, else the pristine set
// shared by every simulation (ro null: rw is complete)
__device__ __forceinline__ const KReqs* ex_req_src(const uint8_t* rw, const uint8_t* ro, const uint64_t* own, int ei) {
  if (ro && !((own[ei >> 6] >> (ei & 63)) & 1)) return reinterpret_cast<const KReqs*>(ro + (size_t)ei * sizeof(KReqs));
  return reinterpret_cast<const KReqs*>(rw + (size_t)ei * sizeof(KReqs));
}

__device__ __forceinline__ void store_merged(KReqs* dst, const ReqView& rv, uint64_t m_v, int W, int KB) {
  const int lane = LANE;
  if (lane < W) dst->vals[lane] = m_v;
  if (lane < KB) {
    dst->gt[lane] = rv.gt[lane];
    dst->lt[lane] = rv.lt[lane];
    dst->minv[lane] = rv.minv[lane];
  }
  if (lane == 0) {
    dst->present = rv.present;
    dst->compl_ = rv.compl_;
    dst->hgt = rv.hgt;
    dst->hlt = rv.hlt;
    dst->hmin = rv.hmin;
  }
}

// Pinned domain of each topology key on a NodeClaim's (merged) requirements: the value ordinal when the key
// is In{one value}, 0xFE when it admits no value, 0xFF otherwise (multi-valued, complement or absent).
__device__ __forceinline__ void store_tcodes(int n_tk, const int32_t* tk_keys, uint8_t* nc_tcode, int stride, const ReqView& rv,
                             uint64_t m_v, int nc) {
  const int lane = LANE;
  for (int j = 0; j < n_tk; j++) {
    const int k = tk_keys[j];
    const uint64_t w = lane_bcast(m_v, k);
    uint8_t code = 0xFF;
    if (((rv.present >> k) & 1) && !((rv.compl_ >> k) & 1))
      code = w == 0 ? 0xFE : (__builtin_popcountll(w) == 1 ? (uint8_t)__builtin_ctzll(w) : 0xFF);
    if (lane == 0) nc_tcode[(size_t)j * stride + nc] = code;
  }
}

// Ordered compaction of per-thread candidate flags into s_list (positions in scan order). Returns count.
template <int NW>
__device__ __forceinline__ int compact_candidates(bool cand, int pos, int32_t* s_list, int32_t* s_wcnt) {
  const int wave = threadIdx.x >> 6, lane = LANE;
  const uint64_t bal = __ballot(cand);
  if (lane == 0) s_wcnt[wave] = __builtin_popcountll(bal);
  __syncthreads();
  int before = 0, total = 0;
  for (int w = 0; w < NW; w++) {
    const int c = s_wcnt[w];
    before += w < wave ? c : 0;
    total += c;
  }
  if (cand) s_list[before + __builtin_popcountll(bal & ((1ull << lane) - 1))] = pos;
  __syncthreads();
  return total;
}

// Same for 4 rounds of positions per thread: round k covers pos0 + k * NT (NT = NW * 64 threads), so for a short
// scan only round 0 is live; one barrier pair for all rounds. s_list holds 4 * NT entries; s_wcnt 4 * NW.
template <int NW>
// tags (bit k: round k's position carries LIST_TAG) mark candidates that may take the append fast path.
#define LIST_TAG 0x40000000
// nc_fail value: the shape-level was merged into the NodeClaim (never equal to a version)
#define NC_MERGED 0x40000000
// Failure memo value of a permanent failure. NodeClaim.Add / ExistingNode.CanAdd failures are monotone: the
// candidate's requirements only narrow (Add intersects), its remaining types only shrink and its requests only
// grow, so once the pod's shape-level fails (taints, Compatible, the type filter, Fits, minValues) it fails for the
// rest of the Solve. The one exception is Compatible's undefined-key rule (the pod requires a custom key the
// candidate does not define yet, and a later merge may define it): such failures keep the candidate's version.
#define NC_NEVER (-3)
#define LIST_POS(e) ((e) & (LIST_TAG - 1))
__device__ __forceinline__ int compact_candidates_x4(uint32_t flags, int pos0, int32_t* s_list, int32_t* s_wcnt,
                                                     uint32_t tags = 0) {
  constexpr int NT = NW * 64;
  const int wave = threadIdx.x >> 6, lane = LANE;
  uint64_t bal[4];
#pragma unroll
  for (int k = 0; k < 4; k++) bal[k] = __ballot((flags >> k) & 1);
  if (lane < 4) s_wcnt[lane * NW + wave] = __builtin_popcountll(bal[lane & 3]);
  __syncthreads();
  int total = 0, before[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int b = total;
    for (int w = 0; w < NW; w++) {
      const int c = s_wcnt[k * NW + w];
      b += w < wave ? c : 0;
      total += c;
    }
    before[k] = b;
  }
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int k = 0; k < 4; k++)
    if ((flags >> k) & 1)
      s_list[before[k] + __builtin_popcountll(bal[k] & lt)] = (pos0 + k * NT) | (((tags >> k) & 1) ? LIST_TAG : 0);
  __syncthreads();
  return total;
}

// LDS atomic min of the first scan position (round k: pos0 + k * NT) whose flag is set, one atomic per wave
// and round (the wave's lowest lane holds its lowest position).
template <int NT>
__device__ __forceinline__ void first_pos_min(uint32_t flags, int pos0, int32_t* dst) {
  for (int k = 0; k < 4; k++) {
    const uint64_t b = __ballot((flags >> k) & 1);
    if (b && LANE == __builtin_ctzll(b)) atomicMin(dst, pos0 + k * NT);
  }
}

// The same two with an explicit entry / position per round (the chunked order's rounds are chunks, not strides).
template <int NW>
__device__ __forceinline__ int compact_candidates_x4e(uint32_t flags, const int* ent, int32_t* s_list, int32_t* s_wcnt,
                                                      uint32_t tags) {
  const int wave = threadIdx.x >> 6, lane = LANE;
  uint64_t bal[4];
#pragma unroll
  for (int k = 0; k < 4; k++) bal[k] = __ballot((flags >> k) & 1);
  if (lane < 4) s_wcnt[lane * NW + wave] = __builtin_popcountll(bal[lane & 3]);
  __syncthreads();
  int total = 0, before[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int b = total;
    for (int w = 0; w < NW; w++) {
      const int c = s_wcnt[k * NW + w];
      b += w < wave ? c : 0;
      total += c;
    }
    before[k] = b;
  }
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int k = 0; k < 4; k++)
    if ((flags >> k) & 1) s_list[before[k] + __builtin_popcountll(bal[k] & lt)] = ent[k] | (((tags >> k) & 1) ? LIST_TAG : 0);
  __syncthreads();
  return total;
}
__device__ __forceinline__ void first_pos_min_e(uint32_t flags, const int* pos, int32_t* dst) {
  for (int k = 0; k < 4; k++) {
    const uint64_t b = __ballot((flags >> k) & 1);
    if (b && LANE == __builtin_ctzll(b)) atomicMin(dst, pos[k]);
  }
}

template <int NW>
__device__ __forceinline__ int first_ok(const int32_t* s_ok) {
  for (int w = 0; w < NW; w++)
    if (s_ok[w]) return w;
  return -1;
}


// sort.Slice(newNodeClaims, len(Pods) asc), exactly as Go's pdqsort_func would permute it, using the
// invariant that between two sort calls at most ONE mutation happened to the (sorted) slice:
//   mut 1: the NodeClaim at position p gained a pod (key +1);  mut 2: a NodeClaim was appended (key 1).
// pdqsort on such input: n <= 12 -> insertionSort (a stable move); n >= 50 with choosePivot's
// increasingHint -> partialInsertionSort performs one swap + two shifts (a stable move) and returns
// true. Every other case (12 < n < 50 with a descent, or a non-increasing hint) replays the full
// pdqsort on one lane. A stable move is a block shift done by the whole workgroup.
// Max allocatable over a NodeClaim's types at creation, for the resources in `rmask`. Its remaining
// types only shrink, so this stays an upper bound: a NodeClaim whose requests + the pod's exceed it for any
// resource cannot take the pod (Fits fails for every remaining type) and the pre-pass skips it.
// With `head`, the new NodeClaim's pre-check record is written as well: headroom = max allocatable - requests (q_lane:
// lane r holds the requests of resource r) for the first four requested resources (INT64_MAX past them), version 0.
// Max of row r of a [R][T] table over the type set X (lane w holds word w of X): lane l reads type 64 i + l for every
// word i, so each word is one coalesced load and the loads of all words are independent (a per-lane walk over the
// word's set bits made every load wait for the previous one: ~64 dependent round trips per resource).
__device__ __forceinline__ int64_t max_over_types(const int64_t* row, uint64_t X, int TW, int T) {
  const int lane = LANE;
  int64_t mx = INT64_MIN;
  for (int i0 = 0; i0 < TW; i0 += 4) {
    int64_t v[4];
    bool in[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = i0 + j;
      const uint64_t w = i < TW ? lane_bcast(X, i) : 0;
      const int t = i * 64 + lane;
      in[j] = ((w >> lane) & 1) && t < T;
      v[j] = in[j] ? row[t] : INT64_MIN;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) mx = v[j] > mx ? v[j] : mx;
  }
  return wave_max_i64(mx);
}

__device__ __forceinline__ void store_maxalloc(const int64_t* alloc, uint64_t X, int T, uint32_t rmask, int64_t* dst,
                                               NcHead* head = nullptr, int64_t q_lane = 0, int32_t taintset = 0) {
  const int lane = LANE;
  int64_t room0 = INT64_MAX, room1 = INT64_MAX, room2 = INT64_MAX, room3 = INT64_MAX;
  int k = 0;
  const int TW = (T + 63) >> 6;
  for (int r = 0; r < KP_NRES; r++) {
    if (!((rmask >> r) & 1)) continue;
    const int64_t mx = max_over_types(alloc + (size_t)r * T, X, TW, T);
    if (lane == 0) dst[r] = mx;
    if (head) {
      const int64_t room = mx - lane_bcast_i64(q_lane, r);
      if (k == 0) room0 = room;
      else if (k == 1) room1 = room;
      else if (k == 2) room2 = room;
      else if (k == 3) room3 = room;
    }
    k++;
  }
  if (head && lane == 0) {
    head->room[0] = room0;
    head->room[1] = room1;
    head->room[2] = room2;
    head->room[3] = room3;
    head->ver = 0;
    head->taintset = taintset;
  }
}

// The k-th (k < 4) set bit of a requested-resource mask, -1 past its last; and the pre-check record as three 16-byte
// loads (headroom 0-1, headroom 2-3 when more than two resources are requested, version + taint set).
__device__ __forceinline__ int kth_res(uint32_t m, int k) {
  for (int i = 0; i < k && m; i++) m &= m - 1;
  return m ? __builtin_ctz(m) : -1;
}
struct HeadView {
  int64_t r0, r1, r2, r3;
  int32_t ver, ts;
};
__device__ __forceinline__ int64_t i64_of(int lo, int hi) { return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo); }
__device__ __forceinline__ HeadView load_head(const NcHead* h, bool four) {
  const int4* p = reinterpret_cast<const int4*>(h);
  const int4 a = p[0], c = p[2];
  int4 b = make_int4(-1, 0x7FFFFFFF, -1, 0x7FFFFFFF);
  if (four) b = p[1];
  return HeadView{i64_of(a.x, a.y), i64_of(a.z, a.w), i64_of(b.x, b.y), i64_of(b.z, b.w), c.x, c.y};
}

// mutation stack (LDS): entries (t, pos) with t and pos increasing bottom to top; the lowest position mutated
// after time `stamp` is the pos of the first entry with t > stamp. On overflow the bottom half is dropped and
// `lost` remembers the newest dropped time: a query older than it answers 0 (conservative).
#define MSTK_CAP 512
__device__ __forceinline__ int mstack_query(const int32_t LDS* stk, int n, int lost, int stamp) {
  if (stamp < lost) return 0;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (stk[2 * m] > stamp) hi = m;
    else lo = m + 1;
  }
  return lo < n ? stk[2 * lo + 1] : INT32_MAX;
}
// one lane; n_ / lost_: the stack's size and lost-time words (LDS control block)
__device__ __forceinline__ void mstack_push(int32_t LDS* stk, int32_t LDS* n_, int32_t LDS* lost_, int t, int pos) {
  int n = *n_;
  while (n > 0 && stk[2 * (n - 1) + 1] >= pos) n--;
  if (n == MSTK_CAP) {
    const int h = MSTK_CAP / 2;
    *lost_ = stk[2 * (h - 1)];
    for (int i = 0; i < 2 * h; i++) stk[i] = stk[2 * h + i];
    n = h;
  }
  stk[2 * n] = t;
  stk[2 * n + 1] = pos;
  *n_ = n + 1;
}

// mstack_query by one wave: 64 stack entries per step (two dependent LDS reads for a full stack instead of nine).
__device__ __forceinline__ int mstack_query_wave(const int32_t LDS* stk, int n, int lost, int stamp) {
  if (UNLIKELY(stamp < lost)) return 0;
  const int lane = LANE;
  int lo = 0, hi = n;  // answer: first entry with t > stamp, in [lo, hi]
  // (every LDS read below is unconditional, at a clamped index, and its value masked after: a load under a lane
  // condition is an exec-masked block with a branch and its own wait)
  while (hi - lo > 64) {
    const int step = (hi - lo + 63) >> 6;
    const int idx = lo + lane * step;
    const bool in = idx < hi;
    const int tv = stk[2 * min(idx, MSTK_CAP - 1)];
    const uint64_t bal = __ballot(in && tv > stamp);
    if (!bal) {
      lo = lo + (__popcll(__ballot(in)) - 1) * step + 1;  // past the last sample taken (< hi)
    } else {
      const int f = __builtin_ctzll(bal);
      if (f == 0) {
        hi = lo;
        break;
      }
      hi = lo + f * step;
      lo = lo + (f - 1) * step + 1;
    }
  }
  if (hi > lo) {
    const int tv = stk[2 * min(lo + lane, MSTK_CAP - 1)];
    const uint64_t bal = __ballot(lo + lane < hi && tv > stamp);
    lo = bal ? lo + __builtin_ctzll(bal) : hi;
  }
  return lo < n ? stk[2 * lo + 1] : INT32_MAX;
}

// first idx in [lo, hi) whose key (npods[ord[idx]]) is >= K (strict: > K) over a non-decreasing range; hi if
// none. One wave: 64 samples per round, so a few rounds of two dependent loads instead of a serial bisection.
template <class P>
__device__ __forceinline__ int wave_key_search(P ord, P npods, int lo, int hi, int K, bool strict) {
  const int lane = LANE;
  while (lo < hi) {
    const int span = hi - lo;
    const int step = span <= 64 ? 1 : (span + 63) >> 6;
    const int idx = lo + lane * step;
    bool ge = false;
    if (idx < hi) {
      const int key = npods[ord[idx]];
      ge = strict ? key > K : key >= K;
    }
    const uint64_t bal = __ballot(ge);
    if (step == 1) return bal ? lo + __builtin_ctzll(bal) : hi;
    if (!bal) {
      lo = lo + (__popcll(__ballot(idx < hi)) - 1) * step + 1;  // past the last sample taken (< hi)
    } else {
      const int f = __builtin_ctzll(bal);
      if (f == 0) return lo;
      hi = lo + f * step;
      lo = lo + (f - 1) * step + 1;
    }
  }
  return lo;
}

// choosePivot(0, n)'s increasingHint for n >= 50, evaluated by one wave: swaps == 0 exactly when each adjacent
// triple (i-1, i, i+1), (j-1, j, j+1), (k-1, k, k+1) is non-decreasing and so are the middles i <= j <= k
// (every order2 then finds !Less(b, a)). Lanes 0..8 load the nine keys together.
template <class P>
__device__ __forceinline__ bool wave_pivot_increasing(P ord, P npods, int n) {
  const int lane = LANE;
  const int t = lane / 3;
  const int mid = (n / 4) * (t + 1);
  int key = 0;
  if (lane < 9) key = npods[ord[mid + (lane % 3) - 1]];
  const int prev = __shfl(key, lane > 0 ? lane - 1 : 0, 64);
  const int midkey_prev = __shfl(key, lane >= 3 ? lane - 3 : 0, 64);
  bool bad = false;
  if (lane < 9 && (lane % 3) != 0 && key < prev) bad = true;        // within a triple
  if (lane < 9 && (lane % 3) == 1 && lane >= 3 && key < midkey_prev) bad = true;  // middles
  return __ballot(bad) == 0;
}

// The literal pdqsort replay (no stable-move shortcut) by wave 0: when keys < 2^11 and ids < 2^20 the wave packs
// (len(Pods) << 20 | id) into ord so that lane 0's comparisons read one word instead of the ord -> npods chain, then
// unpacks; Less compares the key field only, so the permutation is the one pdqsort_func gives on (ord, npods).
template <class P>
struct NCSortPacked {
  P v;
  __device__ bool Less(int i, int j) const { return ((uint32_t)v[i] >> 20) < ((uint32_t)v[j] >> 20); }
  __device__ void Swap(int i, int j) const {
    const int32_t t = v[i];
    v[i] = v[j];
    v[j] = t;
  }
};
template <class P>
__device__ void slow_sort_wave(P ord, P npods, int n) {
  const int lane = LANE;
  int kmax = 0, imax = 0;
  for (int i = lane; i < n; i += 64) {
    const int id = ord[i];
    kmax = max(kmax, npods[id]);
    imax = max(imax, id);
  }
  kmax = -wave_min_i32(-kmax);
  imax = -wave_min_i32(-imax);
  if (kmax < 2048 && imax < (1 << 20)) {
    for (int i = lane; i < n; i += 64) {
      const int id = ord[i];
      ord[i] = (npods[id] << 20) | id;
    }
    wave_sync();
    if (lane == 0) go_sort_slice(NCSortPacked<P>{ord}, n);
    wave_sync();
    for (int i = lane; i < n; i += 64) ord[i] &= (1 << 20) - 1;
  } else {
    if (lane == 0) go_sort_slice(NCSortT<P>{ord, npods}, n);
  }
  wave_sync();
}

#define DBG_SERIAL 0
#define SH_PER_GLB 8  // stable-move shift: words per thread on the global order arrays
#ifndef SORT_DIAG
#define SORT_DIAG 0  // diagnostic: the full path's sort split (decision / shift cycles, shifted entries, modes) in stats[25..30]
#endif
#ifndef EX_DIAG
#define EX_DIAG 0  // diagnostic: the existing-node scan (range, scanned, cursor clamp, scans, cycles, placed) in stats[25..30]
#endif
#ifndef FX_DIAG
#define FX_DIAG 0  // diagnostic: the fast lane's existing-node scans (scans, rounds, placed, skipped, failed, bailed) in stats[25..30]
#endif
__shared__ uint64_t g_sdiag[6];
template <int NT, class P>
__device__ void sort_newnodeclaims(P ord, P npods, int n, int mut, int p, int32_t* s_ctl, uint64_t* slow = nullptr) {
  const int tid = threadIdx.x;
  const uint64_t sd0 = SORT_DIAG ? __builtin_amdgcn_s_memtime() : 0;
  // s_ctl[7]: 0 nothing, 1 shift-left block (p+1..q-1 -> p..q-2, elem -> q-1), 2 shift-right (q..n-2 -> q+1..n-1,
  // elem -> q), 3 slow path; s_ctl[8..9]: q / elem. Decided by wave 0 (lane-parallel searches).
  if (tid < 64) {
    int mode = 0, q = 0;
    NCSortT<P> S{ord, npods};
    if (mut == 1 && p + 1 < n && S.Less(p + 1, p)) {
      mode = 1;
    } else if (mut == 2 && n >= 2 && S.Less(n - 1, n - 2)) {
      mode = 2;
    }
    if (mode) {
      bool fast = n <= 12;
      if (!fast && n >= 50) {
        if (DBG_SERIAL) {
          int hint = 0;
          if (tid == 0) {
            DevPDQ<NCSortT<P>> PQ{S};
            PQ.choosePivot(0, n, &hint);
          }
          hint = __shfl(hint, 0, 64);
          const bool f2 = wave_pivot_increasing(ord, npods, n);
          if (tid == 0 && f2 != (hint == 0)) printf("HINT MISMATCH n=%d p=%d mut=%d\n", n, p, mut);
          fast = hint == 0;
        } else {
          fast = wave_pivot_increasing(ord, npods, n);
        }
      }
      if (!fast) {
        mode = 3;
      } else if (mode == 1) {  // first q > p with key[q] >= key[p]
        q = wave_key_search(ord, npods, p + 1, n, npods[ord[p]], false);
        if (DBG_SERIAL && tid == 0) {
          const int K = npods[ord[p]];
          int lo = p + 1, hi = n;
          while (lo < hi) { const int m = (lo + hi) >> 1; if (npods[ord[m]] >= K) hi = m; else lo = m + 1; }
          if (lo != q) {
            printf("Q1 MISMATCH n=%d p=%d q=%d lo=%d K=%d\n", n, p, q, lo, K);
            for (int i = p; i < n; i++) printf("k[%d]=%d ", i, npods[ord[i]]);
            printf("\n");
          }
        }
      } else {  // first q with key[q] > key of the appended element (in the sorted prefix [0, n-1))
        q = wave_key_search(ord, npods, 0, n - 1, npods[ord[n - 1]], true);
      }
    }
    if (mode == 3) {
      slow_sort_wave(ord, npods, n);
      if (tid == 0 && slow) slow[0] += 1;
    }
    if (tid == 0) {
      // lowest sorted position whose NodeClaim changed or moved since the last sort (cursor clamp)
      s_ctl[16] = mode == 3 ? 0 : (mut == 1 ? p : (mut == 2 ? (mode == 2 ? q : n - 1) : -1));
      s_ctl[7] = mode;
      s_ctl[8] = q;
      s_ctl[9] = mode == 1 ? ord[p] : (mode == 2 ? ord[n - 1] : 0);
    }
  }
  __syncthreads();
  const int mode = s_ctl[7], q = s_ctl[8], elem = s_ctl[9];
  const uint64_t sd1 = SORT_DIAG ? __builtin_amdgcn_s_memtime() : 0;
  // shifts: SH_PER entries per thread between two barriers (a spilled order array shifts thousands of entries in
  // global memory: the loads of a step are in flight together, and each step costs a load and a store round trip)
  constexpr int SH_PER = std::is_same<P, GlbI32>::value ? SH_PER_GLB : 8;
  if (mode == 1) {
    const int c = q - 1 - p;  // elements p+1..q-1 move left by one
    for (int off = 0; off < c; off += NT * SH_PER) {
      int v[SH_PER];
#pragma unroll
      for (int j = 0; j < SH_PER; j++) {
        const int i = off + j * NT + tid;
        v[j] = i < c ? ord[p + 1 + i] : 0;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SH_PER; j++) {
        const int i = off + j * NT + tid;
        if (i < c) ord[p + i] = v[j];
      }
      __syncthreads();
    }
    if (tid == 0) ord[q - 1] = elem;
  } else if (mode == 2) {
    const int c = n - 1 - q;  // elements q..n-2 move right by one (process from the top down)
    for (int off = 0; off < c; off += NT * SH_PER) {
      int v[SH_PER];
#pragma unroll
      for (int j = 0; j < SH_PER; j++) {
        const int i = c - 1 - (off + j * NT + tid);
        v[j] = i >= 0 ? ord[q + i] : 0;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < SH_PER; j++) {
        const int i = c - 1 - (off + j * NT + tid);
        if (i >= 0) ord[q + i + 1] = v[j];
      }
      __syncthreads();
    }
    if (tid == 0) ord[q] = elem;
  }
  __syncthreads();
  if (SORT_DIAG && !EX_DIAG && tid == 0) {
    g_sdiag[0] += sd1 - sd0;
    g_sdiag[1] += __builtin_amdgcn_s_memtime() - sd1;
    g_sdiag[2] += mode == 1 ? q - 1 - p : mode == 2 ? n - 1 - q : 0;
    if (mode) g_sdiag[2 + mode] += 1;
  }
  if (DBG_SERIAL && tid == 0) {
    for (int i = 1; i < n; i++)
      if (npods[ord[i]] < npods[ord[i - 1]]) {
        if (s_ctl[30] != 12345) printf("UNSORTED after mode=%d mut=%d p=%d q=%d n=%d at %d\n", mode, mut, p, q, n, i);
        s_ctl[30] = 12345;
        break;
      }
  }
  __syncthreads();
}

// sort_newnodeclaims executed by ONE wave (the fast lane): the same decisions (stable move when pdqsort would
// perform one, else the literal pdqsort on lane 0), block shifts by 64 lanes with wave-level ordering only.
// Returns the lowest sorted position whose NodeClaim changed or moved (-1: none), as s_ctl[16] would hold.
// max_shift: a stable move shifting more than this many entries (or a literal pdqsort) is left undone and -2 is
// returned, so that the caller hands the pod to the full path (256 lanes per shift step, pdqsort included).
template <class P>
__device__ __forceinline__ int sort_newnodeclaims_wave(P ord, P npods, int n, int mut, int p, int max_shift,
                                                       uint64_t* slow = nullptr) {
  const int lane = LANE;
  int mode = 0, q = 0;
  NCSortT<P> S{ord, npods};
  if (mut == 1 && p + 1 < n && S.Less(p + 1, p)) {
    mode = 1;
  } else if (mut == 2 && n >= 2 && S.Less(n - 1, n - 2)) {
    mode = 2;
  }
  if (mode) {
    bool fast = n <= 12;
    if (!fast && n >= 50) fast = wave_pivot_increasing(ord, npods, n);
    if (!fast) mode = 3;
    else if (mode == 1) q = wave_key_search(ord, npods, p + 1, n, npods[ord[p]], false);
    else q = wave_key_search(ord, npods, 0, n - 1, npods[ord[n - 1]], true);
  }
  if ((mode == 3 && n > max_shift) || (mode == 1 && q - 1 - p > max_shift) || (mode == 2 && n - 1 - q > max_shift))
    return -2;
  const int low = mode == 3 ? 0 : (mut == 1 ? p : (mut == 2 ? (mode == 2 ? q : n - 1) : -1));
  if (mode == 3) {
    slow_sort_wave(ord, npods, n);
    if (lane == 0 && slow) slow[0] += 1;
  } else if (mode == 1) {
    const int elem = ord[p];
    const int c = q - 1 - p;  // elements p+1..q-1 move left by one
    for (int off = 0; off < c; off += 64) {
      const int i = off + lane;
      const int v = i < c ? ord[p + 1 + i] : 0;
      wave_sync();
      if (i < c) ord[p + i] = v;
    }
    wave_sync();
    if (lane == 0) ord[q - 1] = elem;
  } else if (mode == 2) {
    const int elem = ord[n - 1];
    const int c = n - 1 - q;  // elements q..n-2 move right by one (top block first)
    for (int off = 0; off < c; off += 64) {
      const int i = c - 1 - (off + lane);
      const int v = i >= 0 ? ord[q + i] : 0;
      wave_sync();
      if (i >= 0) ord[q + i + 1] = v;
    }
    wave_sync();
    if (lane == 0) ord[q] = elem;
  }
  wave_sync();
  return low;
}


// Topology.Record of a commit on one node (existing position or NodeClaim id `node`, hcnt / tcode rows of `stride`),
// as the full path's: recorded group i on lane i (rec_list[rec_b + i]; the first 64 prefetched in g0 / aux0, the lanes
// past rec_n repeating the last entry); counted when the group is live and its filter admits the node's taint set
// tsx. A hostname group bumps the node's saturating u8 count; a dictionary key counts once the node holds one value
// of it (value code < 64). Every read is unconditional (the hostname count or the value code through one selected
// row pointer, then the group's count and registered mask): two round trips, the stores masked after.
__device__ __forceinline__ void record_node(int rec_n, int rec_b, int g0, int aux0, int tsx, const int32_t* rec_list,
                                            const int32_t* rec_auxv, const int32_t* tg_live,
                                            const uint64_t* tg_filt_tol, const uint8_t* tcode, uint8_t* hcnt,
                                            size_t stride, int node, int32_t* tg_cnt, uint64_t* tg_reg) {
  const int lane = LANE;
  for (int i0 = 0; i0 < rec_n; i0 += 64) {
    const int ri = i0 + lane;
    int g = g0, aux = aux0;
    if (i0) {  // (past the 64 prefetched; uniform branch)
      const int rc = rec_b + min(ri, rec_n - 1);
      g = rec_list[rc], aux = rec_auxv[rc];
    }
    const int live = tg_live[g];
    const uint64_t ftol = tg_filt_tol[g];
    const uint8_t GLB* src = aux >= 0 ? (const uint8_t GLB*)hcnt + (size_t)aux * stride + node
                                      : (const uint8_t GLB*)tcode + (size_t)(-1 - aux) * stride + node;
    const uint32_t b0 = *src;  // the hostname count (255: an unregistered domain), or the node's value code
    const int cnt0 = ((const int32_t GLB*)tg_cnt)[(size_t)g * 64 + (b0 & 63)];
    const uint64_t reg0 = ((const uint64_t GLB*)tg_reg)[g];
    if (ri < rec_n && live && ((ftol >> tsx) & 1)) {
      if (aux >= 0) {
        hcnt[(size_t)aux * stride + node] = b0 == 255 ? 1 : b0 < 254 ? b0 + 1 : 254;
        tg_reg[g] = 1;
      } else if (b0 < 64) {
        tg_cnt[(size_t)g * 64 + b0] = cnt0 + 1;
        tg_reg[g] = reg0 | (1ull << b0);
      }
    }
  }
}

// record_node in two halves for a commit of at most 64 recorded groups: the reads that do not depend on the commit
// (liveness, taint filter, registered mask, the node's hostname count or value code) issued ahead of the commit's
// stores, so that their wait does not also drain those stores; the group's count (indexed by the code) after.
struct RecRead {
  uint64_t reg0;
  uint32_t b0;
  bool ok;
};
__device__ __forceinline__ RecRead record_read(int rec_n, int g, int aux, int tsx, const int32_t* tg_live,
                                               const uint64_t* tg_filt_tol, const uint8_t* tcode, const uint8_t* hcnt,
                                               size_t stride, int node, const uint64_t* tg_reg) {
  const int lane = LANE;
  const int live = ((const int32_t GLB*)tg_live)[g];
  const uint64_t ftol = ((const uint64_t GLB*)tg_filt_tol)[g];
  const uint8_t GLB* src = aux >= 0 ? (const uint8_t GLB*)hcnt + (size_t)aux * stride + node
                                    : (const uint8_t GLB*)tcode + (size_t)(-1 - aux) * stride + node;
  RecRead r;
  r.b0 = *src;
  r.reg0 = ((const uint64_t GLB*)tg_reg)[g];
  r.ok = lane < rec_n && live && ((ftol >> tsx) & 1);
  return r;
}
__device__ __forceinline__ void record_write(const RecRead& r, int g, int aux, uint8_t* hcnt, size_t stride, int node,
                                             int32_t* tg_cnt, uint64_t* tg_reg) {
  const uint32_t b0 = r.b0;
  const int cnt0 = ((const int32_t GLB*)tg_cnt)[(size_t)g * 64 + (b0 & 63)];
  if (r.ok) {
    if (aux >= 0) {
      hcnt[(size_t)aux * stride + node] = b0 == 255 ? 1 : b0 < 254 ? b0 + 1 : 254;
      tg_reg[g] = 1;
    } else if (b0 < 64) {
      tg_cnt[(size_t)g * 64 + b0] = cnt0 + 1;
      tg_reg[g] = r.reg0 | (1ull << b0);
    }
  }
}

// sort.Slice replay after NodeClaim.Add at sorted position p (pending mutation 1), the common case in one batch:
// lanes read ord[p..p+63] and, for pdqsort's choosePivot, the nine sampled positions, then their keys (two dependent
// LDS reads in all). When pdqsort would do a stable move (n <= 12: insertion sort; n >= 50 with increasingHint:
// partialInsertionSort) and the moved NodeClaim's new place is within the window, the ids already in registers
// are written back shifted. Returns the cursor clamp (p), or -2: the general replay (sort_newnodeclaims_wave).
__device__ __forceinline__ int sort_mut1_window(LdsI32 ord, LdsI32 npods, int n, int p, int cap,
                                                 bool* moved = nullptr) {
  const int lane = LANE;
  const int i = p + lane;
  const int t = lane / 3;
  const int pidx = (n / 4) * (t + 1) + (lane % 3) - 1;  // choosePivot's samples (lanes 0..8, n >= 50)
  const bool piv = lane < 9 && n >= 50;
  // unconditional reads at clamped indices (cap: the arrays' length), values masked after: no exec-masked blocks
  const int id_r = ord[min(i, cap - 1)];
  const int pid_r = ord[piv ? pidx : 0];
  const int id = i < n ? id_r : 0;
  const int pid = piv ? pid_r : 0;
  const int key_r = npods[id], pkey_r = npods[pid];
  const int key = i < n ? key_r : INT32_MAX;
  const int pkey = piv ? pkey_r : 0;
  const int K = __builtin_amdgcn_readfirstlane(key);  // npods of the mutated NodeClaim (position p)
  const uint64_t less = __ballot(lane > 0 && i < n && key < K);
  if (LIKELY(!((less >> 1) & 1))) return p;  // Less(p + 1, p) false: sort.Slice leaves the order as it is
  if (moved) *moved = true;
  if (n > 12) {
    if (n < 50) return -2;
    const int prev = __shfl(pkey, lane > 0 ? lane - 1 : 0, 64);
    const int midprev = __shfl(pkey, lane >= 3 ? lane - 3 : 0, 64);
    const bool bad = piv && (((lane % 3) != 0 && pkey < prev) || ((lane % 3) == 1 && lane >= 3 && pkey < midprev));
    if (__ballot(bad)) return -2;  // not increasingHint: the literal pdqsort
  }
  const uint64_t ge = __ballot(lane > 0 && (i >= n || key >= K));
  if (!ge) return -2;  // the tie run continues past the window
  const int q = __builtin_ctzll(ge);  // elements p+1 .. p+q-1 move left by one, the mutated one lands at p+q-1
  wave_sync();
  if (lane >= 1 && lane < q) ord[i - 1] = id;
  const int elem = __builtin_amdgcn_readfirstlane(id);
  if (lane == 0) ord[p + q - 1] = elem;
  wave_sync();
  return p;
}

// mutation stack push (mstack_push) with the stack's size / lost time / clock in registers (uniform)
__device__ __forceinline__ void mstack_push_reg(int32_t LDS* stk, int& n, int& lost, int t, int pos) {
  const int lane = LANE;
  // pop the entries whose position is >= pos: positions increase bottom to top, so they are a suffix, found 64 entries
  // per LDS read (one read in the common case instead of one dependent read per popped entry)
  for (;;) {
    const int base = max(0, n - 64);
    const int j = base + lane;
    const int pv = stk[2 * min(j, MSTK_CAP - 1) + 1];
    const uint64_t ge = __ballot(j < n && pv >= pos);
    if (!ge) break;                         // nothing to pop
    n = base + __builtin_ctzll(ge);         // the suffix starts here ...
    if (n > base || base == 0) break;       // ... unless it may reach below this window
  }
  if (n == MSTK_CAP) {
    const int h = MSTK_CAP / 2;
    lost = stk[2 * (h - 1)];
    for (int i = lane; i < 2 * h; i += 64) {
      const int v = stk[2 * h + i];
      wave_sync();
      stk[i] = v;
    }
    wave_sync();
    n = h;
  }
  if (lane == 0) {
    stk[2 * n] = t;
    stk[2 * n + 1] = pos;
  }
  n++;
  wave_sync();
}

// ---- the spilled newNodeClaims order as chunks ------------------------------------------------------------------
// Past the LDS sort capacity the sorted order is a sequence of chunks of at most 64 NodeClaims: one global block per
// chunk (ids and len(Pods) in order, ChkBlk), and a directory in LDS (the LDS sort arrays' space): per chunk its block,
// count and last key, and the logical position of its first entry. sort.Slice's stable move (one NodeClaim from its
// place to the end of its key run, or an appended one into place) then rewrites at most two blocks and a range of
// directory start positions instead of shifting every entry between the two places (5.3k entries per pop on config 5
// with the flat array). Each block carries the epoch of its last insertion: a shape-level's pre-pass marks a chunk
// whose NodeClaims all fail it permanently (headroom, taints, host ports, NEVER in the failure memo: properties that
// only get worse as a NodeClaim takes pods), and skips it while no NodeClaim entered the block since.
// Every helper here is executed by one wave with uniform arguments.
#define CHK_FILL 48        // entries per chunk when the directory is (re)built
#define CHK_KEY_MAX 8191   // len(Pods) the directory's last-key field holds; more: the flat order
struct ChkDir {
  int32_t LDS* start;   // [CHK_MAXC] logical position of the chunk's first entry
  uint32_t LDS* info;   // [CHK_MAXC] block | count << 12 | last key << 19
  int32_t LDS* bep;     // [CHK_MAXC] per block id: epoch of its last insertion
  uint16_t LDS* freel;  // [CHK_MAXC] free block ids (stack)
};
__device__ __forceinline__ ChkDir chk_dir(int32_t LDS* s) {
  return ChkDir{s, (uint32_t LDS*)(s + CHK_MAXC), s + 2 * CHK_MAXC, (uint16_t LDS*)(s + 3 * CHK_MAXC)};
}
__device__ __forceinline__ int ci_blk(uint32_t v) { return (int)(v & 0xFFF); }
__device__ __forceinline__ int ci_cnt(uint32_t v) { return (int)((v >> 12) & 0x7F); }
__device__ __forceinline__ int ci_last(uint32_t v) { return (int)(v >> 19); }
__device__ __forceinline__ uint32_t ci_make(int b, int cnt, int last) {
  return (uint32_t)b | ((uint32_t)cnt << 12) | ((uint32_t)min(last, CHK_KEY_MAX) << 19);
}
struct ChkCtl {
  int32_t nch, nfree, epoch, maxc;  // chunks, free blocks, insertion epoch counter, directory limit
  int32_t nch_peak, splits, removals, rebuilds;  // diagnostics
};
__shared__ ChkCtl g_chk;

// first index in [lo, hi) where the monotone predicate (false ... true) holds; hi if none. 64 samples per round.
template <class Pred>
__device__ __forceinline__ int wave_first_true(int lo, int hi, Pred pred) {
  const int lane = LANE;
  while (lo < hi) {
    const int span = hi - lo;
    const int step = span <= 64 ? 1 : (span + 63) >> 6;
    const int idx = lo + lane * step;
    const uint64_t bal = __ballot(idx < hi && pred(idx));
    if (step == 1) return bal ? lo + __builtin_ctzll(bal) : hi;
    if (!bal) {
      lo = lo + (__popcll(__ballot(idx < hi)) - 1) * step + 1;
    } else {
      const int f = __builtin_ctzll(bal);
      if (f == 0) return lo;
      hi = lo + f * step;
      lo = lo + (f - 1) * step + 1;
    }
  }
  return lo;
}
// chunk holding logical position pos (< n)
__device__ __forceinline__ int chk_find(const ChkDir& d, int nch, int pos) {
  return wave_first_true(0, nch, [&](int c) { return d.start[c] > pos; }) - 1;
}
// the same by one lane (its own pos)
__device__ __forceinline__ int chk_find_lane(const ChkDir& d, int nch, int pos) {
  int lo = 0, hi = nch;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (d.start[m] > pos) hi = m;
    else lo = m + 1;
  }
  return lo - 1;
}
__device__ __forceinline__ void chk_load(const ChkBlk* B, int b, int cnt, int& id, int& key) {
  const int lane = LANE;
  const int id_r = B[b].id[lane], key_r = B[b].key[lane];  // (unconditional: a block holds 64 entries)
  id = lane < cnt ? id_r : -1;
  key = lane < cnt ? key_r : INT32_MAX;
}
__device__ __forceinline__ void chk_store(ChkBlk* B, int b, int cnt, int id, int key) {
  const int lane = LANE;
  if (lane < cnt) {
    B[b].id[lane] = id;
    B[b].key[lane] = key;
  }
}
// directory entries [i, nch) move up by one (room at i) / [i + 1, nch) down by one (entry i removed)
__device__ void chk_dir_open(const ChkDir& d, int nch, int i) {
  const int lane = LANE;
  for (int top = nch; top > i; top -= 64) {
    const int j = top - 1 - lane;
    const bool act = j >= i;
    const int s = act ? d.start[j] : 0;
    const uint32_t v = act ? d.info[j] : 0;
    wave_sync();
    if (act) {
      d.start[j + 1] = s;
      d.info[j + 1] = v;
    }
    wave_sync();
  }
}
__device__ void chk_dir_close(const ChkDir& d, int nch, int i) {
  const int lane = LANE;
  for (int b = i + 1; b < nch; b += 64) {
    const int j = b + lane;
    const bool act = j < nch;
    const int s = act ? d.start[j] : 0;
    const uint32_t v = act ? d.info[j] : 0;
    wave_sync();
    if (act) {
      d.start[j - 1] = s;
      d.info[j - 1] = v;
    }
    wave_sync();
  }
}

// (Re)builds the directory from a sorted flat order (order[i], npods[id]) of n entries, CHK_FILL per chunk; every block
// gets a new epoch. false: it does not fit (the caller keeps the flat order).
__device__ bool chk_build(const ChkDir& d, ChkCtl LDS* C, ChkBlk* B, const int32_t* order, const int32_t* npods, int n) {
  const int lane = LANE;
  const int nch = (n + CHK_FILL - 1) / CHK_FILL;
  const int maxc = U(C->maxc);
  if (nch > maxc) return false;
  int kmax = 0;
  for (int c = lane; c < nch; c += 64) {
    const int cnt = min(CHK_FILL, n - c * CHK_FILL);
    kmax = max(kmax, npods[order[c * CHK_FILL + cnt - 1]]);
  }
  kmax = -wave_min_i32(-kmax);
  if (kmax > CHK_KEY_MAX) return false;
  const int ep = U(C->epoch) + 1;
  for (int i = lane; i < n; i += 64) {
    const int id = order[i];
    const int c = i / CHK_FILL, s = i - c * CHK_FILL;
    B[c].id[s] = id;
    B[c].key[s] = npods[id];
  }
  for (int c = lane; c < nch; c += 64) {
    const int cnt = min(CHK_FILL, n - c * CHK_FILL);
    d.start[c] = c * CHK_FILL;
    d.info[c] = ci_make(c, cnt, npods[order[c * CHK_FILL + cnt - 1]]);
  }
  for (int b = lane; b < maxc; b += 64) {
    d.bep[b] = ep;
    if (b >= nch) d.freel[b - nch] = (uint16_t)b;
  }
  if (lane == 0) {
    C->nch = nch;
    C->nfree = maxc - nch;
    C->epoch = ep;
    C->nch_peak = max(C->nch_peak, nch);
    C->rebuilds += 1;
  }
  wave_sync();
  return true;
}

// The flat order (order / npods) from the chunks; `n` entries.
__device__ void chk_materialize(const ChkDir& d, ChkCtl LDS* C, const ChkBlk* B, int32_t* order, int32_t* npods) {
  const int lane = LANE;
  const int nch = U(C->nch);
  for (int c = 0; c < nch; c++) {
    const uint32_t v = d.info[c];
    const int cnt = ci_cnt(v), b = ci_blk(v), s0 = d.start[c];
    if (lane < cnt) {
      const int id = B[b].id[lane];
      order[s0 + lane] = id;
      npods[id] = B[b].key[lane];
    }
  }
  wave_sync();
}

// Appends NodeClaim e (len(Pods) key) at the end of the order. false: the directory is full (no change made).
__device__ bool chk_append(const ChkDir& d, ChkCtl LDS* C, ChkBlk* B, int e, int key) {
  const int lane = LANE;
  const int nch = U(C->nch);
  if (nch > 0) {
    const uint32_t v = d.info[nch - 1];
    const int cnt = ci_cnt(v), b = ci_blk(v);
    if (cnt < 64) {
      const int ep = U(C->epoch) + 1;
      if (lane == 0) {
        B[b].id[cnt] = e;
        B[b].key[cnt] = key;
        d.info[nch - 1] = ci_make(b, cnt + 1, key);
        d.bep[b] = ep;
        C->epoch = ep;
      }
      wave_sync();
      return true;
    }
  }
  if (nch >= U(C->maxc) || U(C->nfree) == 0) return false;
  const int nf = U(C->nfree) - 1;
  const int b = d.freel[nf];
  const int s0 = nch ? d.start[nch - 1] + ci_cnt(d.info[nch - 1]) : 0;
  const int ep = U(C->epoch) + 1;
  if (lane == 0) {
    B[b].id[0] = e;
    B[b].key[0] = key;
    d.start[nch] = s0;
    d.info[nch] = ci_make(b, 1, key);
    d.bep[b] = ep;
    C->epoch = ep;
    C->nfree = nf;
    C->nch = nch + 1;
    C->nch_peak = max(C->nch_peak, nch + 1);
  }
  wave_sync();
  return true;
}

// Moves the entry at (cf, sf) to just before the entry at (cx, sx) (cx < 0: to the end of the order), keeping every
// other entry's relative order. (idf, keyf): the source chunk's contents, as its lanes hold them; (lc, lid, lkey): chunk
// lc's contents when lc >= 0 (the replay's search loaded it), so that no block is read twice. An entry landing at a
// chunk's end is one store (the block is not read). false: the target chunk is full and the directory cannot take a
// split (no change made).
__device__ bool chk_move(const ChkDir& d, ChkCtl LDS* C, ChkBlk* B, int cf, int sf, int idf, int keyf, int cx, int sx,
                         int lc, int lid, int lkey) {
  const int lane = LANE;
  int nch = U(C->nch);
  const uint32_t vf = d.info[cf];
  const int bf = ci_blk(vf), nf = ci_cnt(vf);
  const int E = __builtin_amdgcn_readlane(idf, sf), KE = __builtin_amdgcn_readlane(keyf, sf);
  int tc, ts;  // insert before slot ts of chunk tc (ts == count: at its end), in the pre-move contents
  if (cx < 0) {
    tc = nch - 1;
    ts = ci_cnt(d.info[tc]);
  } else {
    tc = cx;
    ts = sx;
  }
  if (ts == 0 && tc > 0) {  // before a chunk's first entry = after the previous chunk's last: no shift there
    const int pc = ci_cnt(d.info[tc - 1]);
    if (pc < 64 || tc - 1 == cf) {
      tc -= 1;
      ts = pc;
    }
  }
  if (tc == cf) {  // within one chunk: remove slot sf, insert at ins (post-removal index)
    const int ins = ts > sf ? ts - 1 : ts;
    int src;
    if (ins >= sf) src = lane < sf ? lane : lane < ins ? lane + 1 : lane == ins ? -1 : lane;
    else src = lane < ins ? lane : lane == ins ? -1 : lane <= sf ? lane - 1 : lane;
    const int sid = __shfl(idf, src < 0 ? 0 : src, 64), skey = __shfl(keyf, src < 0 ? 0 : src, 64);
    const int nid = src < 0 ? E : sid, nkey = src < 0 ? KE : skey;
    chk_store(B, bf, nf, nid, nkey);
    const int last = __builtin_amdgcn_readlane(nkey, nf - 1);
    if (lane == 0) d.info[cf] = ci_make(bf, nf, last);
    wave_sync();
    return true;
  }
  uint32_t vt = d.info[tc];
  int bt = ci_blk(vt), nt = ci_cnt(vt);
  const bool append = ts == nt && nt < 64;  // at the target chunk's end: its contents are not needed
  int idt = 0, keyt = 0;
  if (!append) {
    if (tc == lc) {
      idt = lid;
      keyt = lkey;
    } else {
      chk_load(B, bt, nt, idt, keyt);
    }
  }
  if (nt == 64) {  // split the target chunk: its upper half into a new block and directory entry tc + 1
    if (nch >= U(C->maxc) || U(C->nfree) == 0) return false;
    const int nfr = U(C->nfree) - 1;
    const int b2 = d.freel[nfr];
    const int ep = U(C->epoch) + 1;
    const int hid = __shfl(idt, (lane + 32) & 63, 64), hkey = __shfl(keyt, (lane + 32) & 63, 64);
    chk_store(B, b2, 32, hid, hkey);
    chk_dir_open(d, nch, tc + 1);
    const int s_lo = d.start[tc];
    if (lane == 0) {
      d.start[tc + 1] = s_lo + 32;
      d.info[tc] = ci_make(bt, 32, __builtin_amdgcn_readlane(keyt, 31));
      d.info[tc + 1] = ci_make(b2, 32, __builtin_amdgcn_readlane(keyt, 63));
      d.bep[b2] = ep;
      C->epoch = ep;
      C->nfree = nfr;
      C->nch = nch + 1;
      C->nch_peak = max(C->nch_peak, nch + 1);
      C->splits += 1;
    }
    wave_sync();
    nch += 1;
    if (cf > tc) cf += 1;
    if (ts > 32) {
      tc += 1;
      ts -= 32;
      bt = b2;
      idt = hid;
      keyt = hkey;
    }
    nt = 32;
  }
  // remove from the source chunk
  {
    const int src = lane < sf ? lane : lane + 1;
    const int nid = __shfl(idf, src & 63, 64), nkey = __shfl(keyf, src & 63, 64);
    chk_store(B, bf, nf - 1, nid, nkey);
    if (lane == 0 && nf > 1) d.info[cf] = ci_make(bf, nf - 1, __builtin_amdgcn_readlane(nkey, nf - 2));
  }
  // insert into the target chunk
  const int ep = U(C->epoch) + 1;
  if (append) {
    if (lane == 0) {
      B[bt].id[nt] = E;
      B[bt].key[nt] = KE;
      d.info[tc] = ci_make(bt, nt + 1, KE);
    }
  } else {
    const int src = lane < ts ? lane : lane - 1;
    const int sid = __shfl(idt, src < 0 ? 0 : src, 64), skey = __shfl(keyt, src < 0 ? 0 : src, 64);
    const int nid = lane == ts ? E : sid, nkey = lane == ts ? KE : skey;
    chk_store(B, bt, nt + 1, nid, nkey);
    const int last = __builtin_amdgcn_readlane(nkey, nt);
    if (lane == 0) d.info[tc] = ci_make(bt, nt + 1, last);
  }
  if (lane == 0) {
    d.bep[bt] = ep;
    C->epoch = ep;
  }
  wave_sync();
  // first positions between the two chunks shift by the moved entry
  if (tc > cf) {
    for (int c = cf + 1 + lane; c <= tc; c += 64) d.start[c] -= 1;
  } else {
    for (int c = tc + 1 + lane; c <= cf; c += 64) d.start[c] += 1;
  }
  wave_sync();
  if (nf == 1) {  // the source chunk emptied: drop its directory entry, free its block
    chk_dir_close(d, nch, cf);
    if (lane == 0) {
      const int nfr = C->nfree;
      d.freel[nfr] = (uint16_t)bf;
      C->nfree = nfr + 1;
      C->nch = nch - 1;
      C->removals += 1;
    }
    wave_sync();
  }
  return true;
}

// sort.Slice(newNodeClaims) replay on the chunked order after one pending mutation (see sort_newnodeclaims): the same
// decisions (stable move when pdqsort makes one, else the literal pdqsort over the materialised flat order, then a
// rebuild). Returns the lowest sorted position whose NodeClaim changed or moved (-1: none); -3: the move does not fit
// the directory (nothing changed; the caller continues on the flat order: chk_materialize, then the flat replay);
// -4: the literal pdqsort ran and the rebuild did not fit (the flat order in order / npods is sorted, low = 0).
// choosePivot's increasingHint (n >= 50) needs no loads here: the order was sorted before the mutation, so an appended
// entry (at n - 1, past every sample) leaves every sampled triple non-decreasing, and a +1 at position p whose
// successor is now smaller breaks exactly the triples holding the pair (p, p + 1): p = m - 1 or p = m for a sample
// middle m = (n / 4) * (t + 1) (wave_pivot_increasing's predicate under that invariant).
// hc / hid / hkey: a chunk whose block the caller holds in registers as it now is (ids and keys, lane values; the
// fast lane's last commit chunk, its key already +1), or hc = -1.
__device__ int chk_sort(const ChkDir& d, ChkCtl LDS* C, ChkBlk* B, int n, int mut, int p, int32_t* order,
                        int32_t* npods, uint64_t* slow, int hc = -1, int hblk = -1, int hid = 0, int hkey = 0) {
  const int lane = LANE;
  if (mut == 0) return -1;
  const int nch = U(C->nch);
  int mode = 0, cf = 0, sf = 0, K = 0;
  int id = -1, key = INT32_MAX, cnt = 0;
  if (mut == 1) {
    cf = chk_find(d, nch, p);
    sf = p - d.start[cf];
    const uint32_t v = d.info[cf];
    cnt = ci_cnt(v);
    if (cf == hc && ci_blk(v) == hblk) {  // the block the commit just updated: no reload
      id = lane < cnt ? hid : -1;
      key = lane < cnt ? hkey : INT32_MAX;
    } else {
      chk_load(B, ci_blk(v), cnt, id, key);
    }
    K = __builtin_amdgcn_readlane(key, sf);
    if (K > CHK_KEY_MAX) return -3;
    if (lane == 0) d.info[cf] = ci_make(ci_blk(v), cnt, __builtin_amdgcn_readlane(key, cnt - 1));  // the commit's +1
    wave_sync();
    int kn = INT32_MAX;
    if (sf + 1 < cnt) kn = __builtin_amdgcn_readlane(key, sf + 1);
    else if (cf + 1 < nch) kn = B[ci_blk(d.info[cf + 1])].key[0];
    if (p + 1 < n && kn < K) mode = 1;
  } else {
    cf = nch - 1;
    const uint32_t v = d.info[cf];
    cnt = ci_cnt(v);
    sf = cnt - 1;
    chk_load(B, ci_blk(v), cnt, id, key);
    K = __builtin_amdgcn_readlane(key, sf);
    int kp = INT32_MIN;
    if (sf >= 1) kp = __builtin_amdgcn_readlane(key, sf - 1);
    else if (nch >= 2) {
      const uint32_t w = d.info[nch - 2];
      kp = B[ci_blk(w)].key[ci_cnt(w) - 1];
    }
    if (n >= 2 && K < kp) mode = 2;
  }
  if (!mode) return mut == 1 ? p : n - 1;
  bool fast = n <= 12;
  if (!fast && n >= 50) {
    fast = true;
    if (mode == 1)
      for (int t = 1; t <= 3; t++) {
        const int m = (n / 4) * t;
        if (p == m - 1 || p == m) fast = false;
      }
  }
  if (!fast) {  // the literal pdqsort over the flat order, then a rebuild
    chk_materialize(d, C, B, order, npods);
    slow_sort_wave((GlbI32)order, (GlbI32)npods, n);
    if (lane == 0 && slow) slow[0] += 1;
    return chk_build(d, C, B, order, npods, n) ? 0 : -4;
  }
  int cx = -1, sx = 0, low, lc = -1, lid = 0, lkey = 0;
  if (mode == 1) {  // q = first position > p with key >= K: within the chunk, else the first later chunk reaching K
    const uint64_t bal = __ballot(lane > sf && lane < cnt && key >= K);
    if (bal) {
      cx = cf;
      sx = __builtin_ctzll(bal);
    } else {
      const int c = wave_first_true(cf + 1, nch, [&](int c) { return ci_last(d.info[c]) >= K; });
      if (c < nch) {
        const uint32_t w = d.info[c];
        chk_load(B, ci_blk(w), ci_cnt(w), lid, lkey);
        lc = cx = c;
        sx = __builtin_ctzll(__ballot(lkey >= K));
      }
    }
    low = p;
  } else {  // q = first position in [0, n - 1) with key > K (the appended entry is the last)
    const int c = wave_first_true(0, nch - 1, [&](int c) { return ci_last(d.info[c]) > K; });
    if (c < nch - 1) {
      const uint32_t w = d.info[c];
      chk_load(B, ci_blk(w), ci_cnt(w), lid, lkey);
      lc = cx = c;
      sx = __builtin_ctzll(__ballot(lane < ci_cnt(w) && lkey > K));
    } else {
      cx = cf;
      sx = __builtin_ctzll(__ballot(lane < sf && key > K));
    }
    low = d.start[cx] + sx;
  }
  if (!chk_move(d, C, B, cf, sf, id, key, cx, sx, lc, lid, lkey)) return -3;
  return low;
}

// ---- solve_kernel's fast lane (wave 0), compiled as its own function ------------------------------------------
// State shared with the kernel lives in LDS at file scope (one solve workgroup per CU); the kernel arguments are
// read through the kernarg segment (scalar loads), so the lane's registers are allocated for this loop alone
// instead of inheriting the full path's pressure (whose spills and copies dominated the per-pod instruction count).
#define KARG __attribute__((address_space(4)))
__shared__ DevDict g_D;
__shared__ int32_t g_ctl[34];  // [32] kp_cancel: pops at the next flag read, [33] 1: cancelled
__shared__ int32_t g_stk[2][2 * MSTK_CAP];  // mutation stacks: [0] in-flight positions, [1] existing positions
__shared__ int64_t g_fitv[FITV_RES * FITV_CAP];  // Fits threshold values of catalogue 0 (CatHdr.fit_slot rows)
__shared__ CatHdr g_hdr[8];                      // catalogue descriptors 0..7
__shared__ int32_t fl_fitj[KP_NRES];             // the fast lane's per-wave scratch (wave 0)
__shared__ RowPtr fl_rl[RL_CAP];
__shared__ CatHdr fl_hdrw;
__shared__ KReqs fl_B;                           // the popped pod's requirements (staged on its first merge)
__shared__ WaveSlots fl_slots;
__shared__ uint32_t fl_scratch[2 * KP_MAX_WORDS];
struct FastState {
  int32_t qw_head, qw_n, qw_next, reserved_;
  int32_t qw_pod[64], qw_shape[64], qw_sl[64], qw_lastlen[64], qw_epoch[64];  // lane i: queue entry qw_head + i
  uint64_t bytes, attempts, scanned, starts, fpods, runpods;
  uint64_t fcyc[16];  // [0..5] phases; [6..13] finer probes (FT_FINE builds, exported in place of stats[16..23])
  uint32_t fbail[8];
};
__shared__ FastState g_fast;

__shared__ uint64_t fl_io[2];  // results of the fast lane's out-of-line helpers
// Rare paths of the fast lane's append attempt as calls: a catalogue id >= 8 (descriptor copied to LDS) and more
// than 4 requested resources (fits_filter); inlined, their registers weigh on every pod (config 2 kernel 211.6 ->
// 206.4 ms out of line, same algorithmic bytes).
__device__ __noinline__ void fl_hdr_fill(uint64_t cats_a, int c_a, int C_a) {
  const DevCatalog* cats = (const DevCatalog*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(cats_a >> 32)) << 32) |
                                               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cats_a));
  hdr_fill_wave((CatHdr LDS*)&fl_hdrw, &cats[U(c_a)], U(C_a));
  wave_sync();
}
__device__ __noinline__ uint64_t fl_fits_filter(int cat_a, uint64_t X0, int64_t q_lane, int32_t j0_lane, uint32_t rmask_a,
                                                uint64_t cats_a) {
  const int cat = U(cat_a);
  const DevDict& D = g_D;
  if (cat >= 8) fl_hdr_fill(cats_a, cat, D.C);
  const CatHdr LDS* H = cat < 8 ? (const CatHdr LDS*)&g_hdr[cat] : (const CatHdr LDS*)&fl_hdrw;
  uint64_t nb = 0;
  const uint64_t X = fits_filter(D, H, X0, q_lane, j0_lane, (const int64_t LDS*)g_fitv, (uint32_t)U((int)rmask_a),
                                 (RowPtr LDS*)fl_rl, &nb, fl_fitj);
  if (LANE == 0) fl_io[1] = nb;
  wave_sync();
  return X;
}

// kp_cancel: the caller's flag in host-mapped memory, read past every cache (system scope)
__device__ __forceinline__ bool cancel_set(const int32_t* flag) {
  // (readfirstlane: every lane reads the same word; without it the atomic load counts as divergent, and a loop that
  // breaks on it is compiled as divergent control flow)
  return flag && __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != 0;
}

// A SolveArgs field from the fast lane's lane table (kt0..kt4: dword 64 k + l in lane l of kt<k>); off is a constant,
// so this is one v_readlane per dword.
// A pointer field is rebuilt as a global-address-space pointer and cast to a generic one: kernel-argument pointers
// point to global memory, which the backend infers for pointers it loads from the kernarg segment but not for lane
// values; through the cast, accesses stay global_* instructions instead of FLAT ones (which also wait on the LDS
// counter).
template <class T>
struct ka_type {
  using type = T;
};
template <class U>
struct ka_type<U*> {
  using type = U GLB*;
};
template <class T>
__device__ __forceinline__ T ka_read(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t k4, unsigned off) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte fields");
  auto rd = [&](unsigned j) -> uint32_t {
    const uint32_t v = j < 64 ? k0 : j < 128 ? k1 : j < 192 ? k2 : j < 256 ? k3 : k4;
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(j & 63));
  };
  if constexpr (sizeof(T) == 8) {
    const uint64_t x = ((uint64_t)rd(off / 4 + 1) << 32) | rd(off / 4);
    typename ka_type<T>::type g;
    __builtin_memcpy(&g, &x, 8);
    return (T)g;
  } else {
    const uint32_t x = rd(off / 4);
    T t;
    __builtin_memcpy(&t, &x, 4);
    return t;
  }
}

// Places popped pods while they need no requirement merge; returns the number placed. A pod it cannot place is
// handed to the full path through g_ctl[6] / g_ctl[26]. Called by wave 0 only. CHK: the order is chunked (the
// directory in s_dyn, see chk_sort): the replay edits the blocks and the scan walks the live chunks, one per round.
// EX: the Solve has existing nodes (addToExistingNode on the wave); without, that code is compiled out, so it costs
// the Solves without existing nodes no registers (measured: 9 % of config 2's kernel when only skipped at run time).
template <bool TOPO, bool CHK, bool EX, bool CONT>
__device__ __noinline__ int fast_lane(uint64_t kargs, int32_t LDS* s_dyn_arg, uint64_t pops_in_arg) {
  // a callee's arguments arrive in VGPRs and count as divergent: made provably uniform here, or every value and
  // branch that depends on them (the whole pod loop) would be compiled as divergent control flow
  // (opaque: every caller passes the kernel's dynamic LDS array, and once the optimiser propagates that into this
  // function each use becomes a scalar load of its offset from the dynamic-LDS table, with an lgkmcnt wait)
  uint32_t s_dyn_off = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)s_dyn_arg);
  asm volatile("" : "+s"(s_dyn_off));
  int32_t LDS* s_dyn = (int32_t LDS*)(uintptr_t)s_dyn_off;
  const uint64_t pops_in = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pops_in_arg >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)pops_in_arg);
  // the kernel's argument block (the kernarg segment pointer is only defined in the kernel itself: it passes it);
  // readfirstlane makes it provably uniform, so field reads are scalar loads
  const uint32_t klo = __builtin_amdgcn_readfirstlane((uint32_t)kargs);
  const uint32_t khi = __builtin_amdgcn_readfirstlane((uint32_t)(kargs >> 32));
  const KARG SolveArgs* A = (const KARG SolveArgs*)(((uint64_t)khi << 32) | klo);
  const DevDict& D = g_D;
  int32_t LDS* s_ctl = (int32_t LDS*)g_ctl;
  auto& s_stk = g_stk;
  FastState LDS* S = (FastState LDS*)&g_fast;
  const int lane = LANE;
  auto hdr = [&](int c) -> const CatHdr LDS* {
    if (c < 8) return (const CatHdr LDS*)&g_hdr[c];
    hdr_fill_wave((CatHdr LDS*)&fl_hdrw, &A->cats[c], D.C);
    wave_sync();
    return (const CatHdr LDS*)&fl_hdrw;
  };
  const uint32_t rmask_all = A->req_res_mask;
  const int rr0 = rmask_all ? __builtin_ctz(rmask_all) : 0;
  const uint32_t rm1 = rmask_all & (rmask_all - 1);
  const int rr1 = rm1 ? __builtin_ctz(rm1) : rr0;
  const uint32_t rr_rest = rm1 & (rm1 - 1);
  // the pre-check record holds the first four requested resources' headroom; more come from requests / maxalloc
  const int rk2 = kth_res(rmask_all, 2), rk3 = kth_res(rmask_all, 3);
  uint32_t rr_b4 = rr_rest;
  for (int i = 0; i < 2 && rr_b4; i++) rr_b4 &= rr_b4 - 1;
  const bool four = rk2 >= 0;
  static_assert(KP_NRES < 63, "lane 63 of the request vector is the zero slot");
  const uint32_t pr_idx = (uint32_t)(rmask_all ? rr0 : 63) | (uint32_t)(rm1 ? rr1 : 63) << 8 |
                          (uint32_t)(rk2 >= 0 ? rk2 : 63) << 16 | (uint32_t)(rk3 >= 0 ? rk3 : 63) << 24;
  uint32_t rrp_all = 0;  // the requested resources (first four as bytes), for pods requesting all of them
  int n_rrp_all = 0;
  for (uint32_t m = rmask_all; m; m &= m - 1) {
    if (n_rrp_all < 4) rrp_all |= (uint32_t)__builtin_ctz(m) << (8 * n_rrp_all);
    n_rrp_all++;
  }
  const uint64_t pop_cap = (uint64_t)A->n_pods * 64 + 65536;
  // the pops this call may still make before the runaway guard (a 32-bit scalar compare per pod)
  const int pop_left = U(pops_in >= pop_cap ? -1 : (int)min<uint64_t>(pop_cap - pops_in, (uint64_t)INT32_MAX));
  // control state in registers for the loop; written back on exit
  int q_head = U(s_ctl[0]), q_len = U(s_ctl[1]), n_ev = U(s_ctl[4]), mut = U(s_ctl[10]), mut_p = U(s_ctl[11]);
  int stk_n = U(s_ctl[12]), stk_t = U(s_ctl[13]), stk_lost = U(s_ctl[20]);  // in-flight mutation stack
  const int n_nc_all = U(s_ctl[2]);
  int epoch = U(s_ctl[3]);  // Queue's lastLen generation (a relaxed memo failure starts a new one)
  const bool in_lds = U(s_ctl[5]) == 1;  // order mode: 1 LDS, 2 chunked, 0 flat global
  int qw_head = U(S->qw_head), qw_n = U(S->qw_n), qw_next = U(S->qw_next);
  int qw_pod = S->qw_pod[lane], qw_shape = S->qw_shape[lane], qw_sl = S->qw_sl[lane], qw_lastlen = S->qw_lastlen[lane],
      qw_epoch = S->qw_epoch[lane];
  // statistics: uniform counters (a lane-0 update of a per-lane 64-bit value costs an exec-masked block per pod: 6 % of
  // config 2's kernel, measured); the positions scanned are n_scan below
  uint64_t bytes = 0, attempts = 0, starts = 0, fcyc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int pops = 0, memo_pops = 0, handoff = -1, fb = -1;
  int chk_next = U(s_ctl[32]);  // kp_cancel: Queue pops (the Solve's total) at which the flag is read next
  // the NodeClaim this call's last append commit wrote, as it wrote it (the next pod usually starts there: reading
  // its lines back right after the stores waits for them to drain): remaining types, requests, threshold indices
  // (lane values), and its pre-check record. Only the fast lane writes NodeClaims during one call.
  int c_nc = -1, c_cat = 0, c_ver = 0, c_ts = 0;
  int cont_w = -1, cont_sl = -1;  // the last commit's position and shape-level when it was an append on c_nc
  uint64_t c_X = 0, c_hm = 0;
  int64_t c_q = 0, c_r0 = 0, c_r1 = 0, c_r2 = 0, c_r3 = 0;
  int32_t c_fj = 0;
  int n_buf = 0, buf_pod = 0, buf_pl = 0;  // placements not yet written (lane i: the i-th)
  // chunked order: the block of the last commit's chunk as the commit left it (ids, keys), for the next replay
  int h_ck = -1, h_blk = -1, h_id = 0, h_key = 0;
  // the append path's byte model as 32-bit event counts, converted on exit (the 64-bit accumulators cost 2.8 % of
  // the loop)
  NbUnits fnb{0, 0, 0};
  uint32_t n_app = 0, n_scan = 0, n_run = 0;
    const bool tmg = A->timing != 0;
    // the argument block as a lane table: dword 64 k + l of SolveArgs in lane l of kt<k>
    static_assert(sizeof(SolveArgs) <= 1280, "SolveArgs outgrew the fast lane's argument table");
    uint32_t kt0, kt1, kt2, kt3, kt4;
    {
      const KARG uint32_t* aw = (const KARG uint32_t*)A;
      const int nw = (int)(sizeof(SolveArgs) / 4);
      kt0 = aw[lane];
      kt1 = 64 + lane < nw ? aw[64 + lane] : 0;
      kt2 = 128 + lane < nw ? aw[128 + lane] : 0;
      kt3 = 192 + lane < nw ? aw[192 + lane] : 0;
      kt4 = 256 + lane < nw ? aw[256 + lane] : 0;
      // landed before the loop: the per-pod asm barrier on these registers then needs no wait (otherwise the
      // waitcnt pass puts a vmcnt(0) at every pod's start, which also waits for the previous pod's stores)
      __builtin_amdgcn_s_waitcnt(0);
    }
#define KA(f) ka_read<decltype(SolveArgs::f)>(kt0, kt1, kt2, kt3, kt4, offsetof(SolveArgs, f))
#define FL_HAS_EX (EX)
    uint64_t ft = tmg ? __builtin_amdgcn_s_memtime() : 0;
#define FTF(i)                                               \
  if (FT_FINE && tmg) {                                      \
    const uint64_t tn_ = __builtin_amdgcn_s_memtime();       \
    fcyc[i] += tn_ - ft;                                     \
    ft = tn_;                                                \
  }
#define FT(i)                                                \
if (!FL_NOTIME && tmg) {                                    \
  const uint64_t tn_ = __builtin_amdgcn_s_memtime();       \
  fcyc[i] += tn_ - ft;                      \
  ft = tn_;                                                \
}
    // next pod's stage data, loaded while the current pod is placed (window offset pf_off; -1: none)
    int pf_off = -1, pf_own = 0, pf_ce0 = 0, pf_ce1 = 0, pf_cur = 0, pf_stamp = 0, prev_sl = -1;
    int pf_stg = 0;  // topology Solves: the next entry's stage record (lane d: dword d of SolveArgs::sl_stage's row)
    int a_cur_prev_pos = 0, a_cur_prev_stamp = 0, a_cex_prev_stamp = 0, a_cex_prev_pos = 0;  // cursors the previous pod stored
    int64_t pf_preq = 0;
    uint64_t pf_tol = 0;
    for (;;) {
      // the argument block's fields are read from the lane table (KA): one or two v_readlane where used, made opaque per
      // pod so that they are not hoisted into SGPRs held across the loop (which spilled into VGPR lanes), and with no
      // scalar load whose lgkmcnt wait would also drain the wave's outstanding LDS operations
      asm volatile("" : "+v"(kt0), "+v"(kt1), "+v"(kt2), "+v"(kt3), "+v"(kt4));
      const int len = q_len;
      const int head = q_head;
      if (UNLIKELY(len <= 0 || pops + memo_pops > pop_left)) break;
      // Queue.Pop from the prefetched window: entries [qw_head, qw_head + qw_n) of the ring were in the queue when
      // the window was read, and nothing rewrites a queued entry (pushes go to the tail) or its pod's level and
      // lastLen stamps while it waits, so lane i's copy of entry qw_head + i stays exact.
      int off = head - qw_head;
      if (off < 0) off += KA(n_pods);
      if (UNLIKELY(off != qw_next || off >= qw_n)) {  // exhausted, or the ring wrapped onto re-pushed entries
        if (KA(cancel) && (int)(pops_in + pops + memo_pops) >= chk_next) {  // ctx.Done(): at most every 1024 pops
          chk_next = (int)(pops_in + pops + memo_pops) + 1024;
          if (cancel_set(KA(cancel))) {
            s_ctl[33] = 1;
            break;
          }
        }
        qw_head = head;
        qw_n = min(64, len);
        off = 0;
        pf_off = -1;
        int qi = head + lane;
        if (qi >= KA(n_pods)) qi -= KA(n_pods);
        if (lane < qw_n) {
          qw_pod = KA(queue)[qi];
          qw_shape = KA(pod_shape)[qw_pod];
          qw_sl = KA(shape_level_base)[qw_shape] + KA(pod_level)[qw_pod];
          qw_lastlen = KA(lastlen)[qw_pod];
          qw_epoch = KA(lastlen_epoch)[qw_pod];
        }
        // wait for the window here, in the rare branch: at the join the compiler would otherwise wait for every
        // outstanding vector-memory operation (the previous pod's stores included) on the common path too
        READY(qw_pod);
        READY(qw_shape);
        READY(qw_sl);
        READY(qw_lastlen);
        READY(qw_epoch);
      }
      qw_next = off + 1;  // only the fast lane pops: the next pop reads the following entry
      const int pod = __builtin_amdgcn_readlane(qw_pod, off);
      if (UNLIKELY(__builtin_amdgcn_readlane(qw_epoch, off) == epoch && __builtin_amdgcn_readlane(qw_lastlen, off) == len))
        break;  // the full path's pop sees the same queue and ends the Solve
      FTF(6);
      const int shape = __builtin_amdgcn_readlane(qw_shape, off);
      const int sl = __builtin_amdgcn_readlane(qw_sl, off);
      // stage: one batch of independent loads (eligibility, requests, tolerations, both first-fit cursors),
      // issued by the previous pod when this entry was next in the window
      int own, ce0, ce1, cur, stamp;
      int64_t preq_lane;
      uint64_t tolmask;
      int stg = 0;  // topology Solves: the shape-level's stage record (eligibility, tolerations, owned / recorded groups)
      if (LIKELY(pf_off == off)) {
        own = U(pf_own), ce0 = U(pf_ce0), ce1 = U(pf_ce1), cur = U(pf_cur), stamp = U(pf_stamp), preq_lane = pf_preq,
        tolmask = U64(pf_tol);
        if (TOPO) {
          stg = pf_stg;
          own = __builtin_amdgcn_readlane(stg, 0);
          tolmask = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(stg, 2) << 32) | (uint32_t)__builtin_amdgcn_readlane(stg, 1);
        }
        if (sl == prev_sl) {  // the previous pod (same shape-level) advanced both cursors after the loads
          cur = a_cur_prev_pos;
          stamp = a_cur_prev_stamp;
          ce0 = a_cex_prev_pos;
          ce1 = a_cex_prev_stamp;
        }
      } else {
        if (!TOPO) own = U(KA(hp_any) && KA(shape_hp_conf)[shape] ? 1 : 0);
        ce0 = U(FL_HAS_EX ? KA(cur_ex)[2 * sl] : 0), ce1 = U(FL_HAS_EX ? KA(cur_ex)[2 * sl + 1] : 0);
        const int64_t pq_r = KA(shape_requests)[(size_t)shape * KP_NRES + min(lane, KP_NRES - 1)];
        preq_lane = lane < KP_NRES ? pq_r : 0;
        if (!TOPO) {
          tolmask = U64(KA(shape_tolerates)[sl]);
        } else {
          stg = KA(sl_stage)[(size_t)sl * 64 + lane];
          own = __builtin_amdgcn_readlane(stg, 0);
          tolmask = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(stg, 2) << 32) | (uint32_t)__builtin_amdgcn_readlane(stg, 1);
        }
        cur = U(KA(cur_nc)[2 * sl]), stamp = U(KA(cur_nc)[2 * sl + 1]);
        READY(preq_lane);
      }
      pf_off = -1;
      if (LIKELY(off + 1 < qw_n)) {  // the next entry's stage loads: in flight while this pod is sorted and placed
        const int nshape = __builtin_amdgcn_readlane(qw_shape, off + 1);
        const int nsl = __builtin_amdgcn_readlane(qw_sl, off + 1);
        if (!TOPO) pf_own = KA(hp_any) && KA(shape_hp_conf)[nshape] ? 1 : 0;
        else pf_stg = KA(sl_stage)[(size_t)nsl * 64 + lane];  // (eligibility and tolerations come from it)
        pf_ce0 = FL_HAS_EX ? KA(cur_ex)[2 * nsl] : 0, pf_ce1 = FL_HAS_EX ? KA(cur_ex)[2 * nsl + 1] : 0;
        const int64_t pq_r = KA(shape_requests)[(size_t)nshape * KP_NRES + min(lane, KP_NRES - 1)];
        pf_preq = lane < KP_NRES ? pq_r : 0;
        if (!TOPO) pf_tol = KA(shape_tolerates)[nsl];
        pf_cur = KA(cur_nc)[2 * nsl], pf_stamp = KA(cur_nc)[2 * nsl + 1];
        pf_off = off + 1;
      }
      prev_sl = sl;
      FTF(7);
      q_head = head + 1 == KA(n_pods) ? 0 : head + 1;
      q_len = len - 1;
      // the unschedulable memo (SolveArgs::sl_fail; chunked orders, where failing pods are many): the pod fails
      // every placement, so after the sort replay below the lane does the full path's failure bookkeeping itself
      const bool memo = CHK && !TOPO && KA(sl_fail)[sl] == n_nc_all;
      bool eligible = own == 0;
      // addToExistingNode's start: the first-fit cursor, clamped by the existing positions mutated since it was stored
      const int ex_start = FL_HAS_EX ? min(ce0, mstack_query_wave((LdsI32)s_stk[1], U(s_ctl[14]), U(s_ctl[21]), ce1))
                                     : 0;
      FT(0);
      if (UNLIKELY(!eligible)) {
        handoff = pod;
        fb = FB_INELIGIBLE;
        break;
      }
      // the first four requested resources' requests (lane 63 holds 0 for an unused slot): no branches
      const int64_t pr0 = lane_bcast_i64(preq_lane, pr_idx & 0xff), pr1 = lane_bcast_i64(preq_lane, (pr_idx >> 8) & 0xff);
      const int64_t pr2 = lane_bcast_i64(preq_lane, (pr_idx >> 16) & 0xff), pr3 = lane_bcast_i64(preq_lane, pr_idx >> 24);
      // the resources this pod requests (chunked orders: many NodeClaims, pools whose pods request few of the
      // resources): Fits on an in-flight NodeClaim only re-tests those (its remaining types already fit its own
      // requests on every other resource, and a zero request leaves them so), and the fifth and later ones'
      // pre-check (requests + pod <= max allocatable) holds trivially for a zero request. Elsewhere the
      // loop-invariant list (the per-pod mask cost 6 % of config 2, measured)
      uint32_t rr_b4p = rr_b4, rrp = rrp_all;  // rrp: the first four as bytes (registers: no indexed array)
      int n_rrp = n_rrp_all;
      if (CHK) {
        const uint32_t pod_rm = rmask_all & (uint32_t)__ballot(lane < KP_NRES && preq_lane > 0);
        if (pod_rm != rmask_all) {
          rr_b4p = rr_b4 & pod_rm, rrp = 0, n_rrp = 0;
          for (uint32_t m = pod_rm; m; m &= m - 1) {
            if (n_rrp < 4) rrp |= (uint32_t)__builtin_ctz(m) << (8 * n_rrp);
            n_rrp++;
          }
        }
      }
      // topology (levels the host marked fast: spread groups only): the owned groups staged in registers, as the full
      // path stages them into s_town / s_tacc (hostname rows: count + self <= maxSkew; dictionary keys: the domains
      // whose count + self - min <= maxSkew)
      int t_n = 0, rec_n = 0, rec_b = 0;
      // the recorded groups of the shape (lane i: the i-th, up to 64), loaded with the stage so that Topology.Record
      // at the commit starts from registers: group, hostname row / key slot, and whether it counts the node's taints
      int r_g = 0, r_aux = 0;
      bool triv = false;  // no requirements at this level: Add on any NodeClaim is Fits alone (the full path's triv)
      int t_key[4] = {0, 0, 0, 0}, t_row[4] = {0, 0, 0, 0}, t_slot[4] = {0, 0, 0, 0}, t_self[4] = {0, 0, 0, 0},
          t_mskew[4] = {0, 0, 0, 0};
      uint64_t t_acc[4] = {0, 0, 0, 0};
      if (TOPO) {  // (every static field from the stage record's registers: the counts are the only loads)
        t_n = __builtin_amdgcn_readlane(stg, 3);
        triv = __builtin_amdgcn_readlane(stg, 4) != 0;
        rec_n = __builtin_amdgcn_readlane(stg, 5);
        rec_b = __builtin_amdgcn_readlane(stg, 6);
        if (rec_n) {  // (the group's liveness and taint filter are read at the commit: no wait here)
          // (the lanes past rec_n repeat the last entry: record_node masks them)
          if (LIKELY(rec_n <= 8)) {  // from the record: lane i takes dwords 48 + 2i and 49 + 2i
            const int src = 48 + 2 * min(lane, rec_n - 1);
            r_g = __builtin_amdgcn_ds_bpermute(src << 2, stg);
            r_aux = __builtin_amdgcn_ds_bpermute((src + 1) << 2, stg);
          } else {  // (uniform branch; reads at clamped lanes, masked after: no exec-masked block)
            const int rl = rec_b + min(lane, rec_n - 1);
            const int g_r = KA(rec_list)[rl], a_r = KA(rec_aux)[rl];
            r_g = g_r, r_aux = a_r;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (j < t_n) {
            const int g = __builtin_amdgcn_readlane(stg, 8 + 8 * j), self = __builtin_amdgcn_readlane(stg, 9 + 8 * j);
            const int key = __builtin_amdgcn_readlane(stg, 10 + 8 * j), mskew = __builtin_amdgcn_readlane(stg, 11 + 8 * j);
            t_key[j] = key, t_row[j] = __builtin_amdgcn_readlane(stg, 13 + 8 * j);
            t_slot[j] = __builtin_amdgcn_readlane(stg, 14 + 8 * j), t_self[j] = self, t_mskew[j] = mskew;
            if (key >= 0) {
              const int c = KA(tg_cnt)[(size_t)g * 64 + lane];
              const uint64_t reg = KA(tg_reg)[g];
              const uint64_t pd = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(stg, 41 + 2 * j) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane(stg, 40 + 2 * j);
              const int mind = __builtin_amdgcn_readlane(stg, 12 + 8 * j);
              const bool sup = ((reg & pd) >> lane) & 1;
              const int mn = wave_min_i32(sup ? c : INT32_MAX);
              const int num = __builtin_popcountll(reg & pd);
              int64_t m = num ? (int64_t)mn : (int64_t)INT32_MAX;
              if (mind > 0 && num < mind) m = 0;
              t_acc[j] = __ballot(((reg >> lane) & 1) && (int64_t)c + self - m <= mskew);
            }
          }
      }
      if (FL_HAS_EX) a_cex_prev_stamp = U(s_ctl[15]);
      bool b_staged = false;  // fl_B holds the pod's requirement set (staged on the first merge)
      // ---- addToExistingNode on the wave: ExistingNode.CanAdd at the lowest position that takes the pod, the
      // full path's checks 64 positions per round (headroom rows, failure memo, static fit, taints, hostname counts,
      // then the zone-like keys' value codes), then the requirement merge on the first candidates. An existing node's
      // labels are single values and its codes were checked against the accepted domains, so the topology narrowing
      // has nothing to narrow. A scan longer than FAST_EX_ROUNDS rounds goes to the full path's 1,024-lane pre-pass.
      if (FL_HAS_EX && ex_start < KA(n_existing) && !memo) {
        const int E = KA(n_existing);
        const bool ex_triv = TOPO ? triv : kreq_at(KA(shape_reqs), sl)->present == 0;
        int ex_pl = -1, ex_ipos = INT32_MAX, rounds = 0;
        bool ex_bail = false;
        // the scan runs over list indices: every position, or (batched simulations) the shape-level's usable list
        const int32_t* ul = KA(ex_ulist);
        int u_base = 0, u_n = E, u_start = ex_start;
        if (ul) {
          u_base = KA(ex_ulist_off)[sl];
          u_n = KA(ex_ulist_off)[sl + 1] - u_base;
          u_start = KA(ex_uidx)[(size_t)sl * E + ex_start];
        }
        if (FX_DIAG && lane == 0) g_sdiag[0] += 1;
        for (int base = u_start; base < u_n && ex_pl < 0; base += 64) {
          if (++rounds > FAST_EX_ROUNDS) {
            ex_bail = true;
            break;
          }
          if (FX_DIAG && lane == 0) g_sdiag[1] += 1;
          const bool valid = base + lane < u_n;
          const int li = min(base + lane, u_n - 1);
          const int ec = ul ? ul[u_base + li] : base + lane;  // (clamped: masked by valid)
          bool cand = false, icand = false;
          int32_t ver = 0, ts = 0;
          {  // every read unconditional at a clamped position, the lanes past E masked after (no exec-masked block)
            const int ecc = min(ec, E - 1);
            // the failure memo: [shape-level][position], or (batched simulations) one entry per list entry
            const int32_t fl = KA(ex_fail)[ul ? (size_t)u_base + li : (size_t)sl * E + ecc];
            ver = KA(ex_ver)[ecc];
            ts = KA(ex_taintset)[ecc];
            const uint8_t sok = KA(ex_static_ok)[ecc];
            const int64_t er0 = KA(ex_room)[ecc], er1 = KA(ex_room)[(size_t)E + ecc];
            const int64_t er2 = four ? KA(ex_room)[2 * (size_t)E + ecc] : INT64_MAX;
            const int64_t er3 = four ? KA(ex_room)[3 * (size_t)E + ecc] : INT64_MAX;
            cand = valid & (er0 >= pr0) & (er1 >= pr1) & (er2 >= pr2) & (er3 >= pr3) & (fl != ver) & (fl != NC_NEVER) &
                   (sok != 0) & (((tolmask >> ts) & 1) != 0);
            if (UNLIKELY(rr_b4p)) {  // a fifth requested resource and beyond
              const int64_t* av = KA(ex_available) + (size_t)ecc * KP_NRES;
              const int64_t* rq = KA(ex_requests) + (size_t)ecc * KP_NRES;
              for (uint32_t rm = rr_b4p; rm; rm &= rm - 1) {
                const int r = __builtin_ctz(rm);
                cand = cand & (rq[r] + lane_bcast_i64(preq_lane, r) <= av[r]);
              }
            }
            if (TOPO && t_n) {
#pragma unroll
              for (int j = 0; j < 4; j++)
                if (j < t_n && t_key[j] < 0)
                  cand = cand & ((int)KA(hcnt_ex)[(size_t)t_row[j] * E + ecc] + t_self[j] <= t_mskew[j]);
              icand = cand;
#pragma unroll
              for (int j = 0; j < 4; j++)
                if (j < t_n && t_key[j] >= 0) {
                  const uint32_t code = KA(ex_tcode)[(size_t)t_slot[j] * E + ecc];
                  cand = cand & (code != 0xFF) & (((t_acc[j] >> (code & 63)) & 1) != 0);
                }
            }
          }
          if (TOPO && t_n && ex_ipos == INT32_MAX) {
            const uint64_t im = __ballot(icand);
            if (im) ex_ipos = __builtin_amdgcn_readlane(ec, __builtin_ctzll(im));
          }
          bytes += (uint64_t)min(64, u_n - base) * (16 * KA(n_req_res) + 13);  // (the full path's model)
          uint64_t cm = __ballot(cand);
          while (cm) {
            const int l = __builtin_ctzll(cm);
            cm &= cm - 1;
            const int ei = __builtin_amdgcn_readlane(ec, l);
            const int32_t verx = __builtin_amdgcn_readlane(ver, l);
            attempts++;
            if (!b_staged && !ex_triv) {  // the pod's requirement set, once per pod
              constexpr int NQ = (int)(sizeof(KReqs) / 8);
              const uint64_t* src = reinterpret_cast<const uint64_t*>(KA(shape_reqs) + (size_t)sl * sizeof(KReqs));
              uint64_t* dstB = reinterpret_cast<uint64_t*>(&fl_B);
              for (int i = lane; i < NQ; i += 64) dstB[i] = src[i];
              wave_sync();
              b_staged = true;
            }
            KReqs* er = reinterpret_cast<KReqs*>(KA(ex_reqs) + (size_t)ei * sizeof(KReqs));
            const KReqs* er_src = ex_req_src(KA(ex_reqs), KA(ex_reqs_ro), KA(ex_own), ei);
            bytes += sizeof(KReqs);
            // a pod without requirements at this level: Compatible holds and Add leaves the node's requirements as
            // they are (nothing to intersect), so neither the merge nor its store is needed
            if (!ex_triv) {
              const CandReq crx = load_cand(D, er_src);
              uint64_t m_v = 0;
              ReqView rv;
              const uint64_t b_negop = KA(shape_negop)[sl];
              const bool mok = merge_compatible(D, crx, (const KReqs*)&fl_B, b_negop, false, m_v, rv,
                                                (WaveSlots*)&fl_slots, vint_global(KA(vint)));
              if (!mok) {  // permanent unless the undefined-key rule failed (no well-known exemption here)
                KA(ex_fail)[ul ? (size_t)u_base + __builtin_amdgcn_readlane(li, l) : (size_t)sl * E + ei] =
                    (fl_B.present & ~crx.P & ~b_negop) == 0 ? NC_NEVER : verx;
                continue;
              }
              // commit: ExistingNode.Add (requirements, requests, headroom rows, version), Topology.Record
              store_merged(er, rv, m_v, D.W, D.KB);
              if (KA(ex_reqs_ro)) KA(ex_own)[ei >> 6] |= 1ull << (ei & 63);  // (uniform: every lane stores the same)
            }
            RecRead rrd{0, 0, false};  // Topology.Record's reads, ahead of the commit's stores (<= 64 groups)
            if (TOPO && rec_n && rec_n <= 64)
              rrd = record_read(rec_n, r_g, r_aux, __builtin_amdgcn_readlane(ts, l), KA(tg_live), KA(tg_filt_tol),
                                KA(ex_tcode), KA(hcnt_ex), (size_t)E, ei, KA(tg_reg));
            {  // requests + pod, the headroom rows of the first four requested resources - pod, version + 1: every
               // lane reads and stores (the lanes past the rows repeat the last row's value), no exec-masked block
              int64_t* rqp = KA(ex_requests) + (size_t)ei * KP_NRES + min(lane, KP_NRES - 1);
              const int64_t rq_n = *rqp + preq_lane;
              const int64_t rq_top = lane_bcast_i64(rq_n, KP_NRES - 1);
              const int hl = min(lane, 3);
              int64_t* hrp = KA(ex_room) + (size_t)hl * E + ei;
              const int64_t d = hl == 0 ? pr0 : hl == 1 ? pr1 : hl == 2 ? pr2 : pr3;
              const int64_t hr_n = *hrp - d;
              *rqp = lane < KP_NRES ? rq_n : rq_top;
              *hrp = hr_n;
              KA(ex_ver)[ei] = verx + 1;
            }
            if (TOPO && rec_n) {
              if (LIKELY(rec_n <= 64))
                record_write(rrd, r_g, r_aux, KA(hcnt_ex), (size_t)E, ei, KA(tg_cnt), KA(tg_reg));
              else
                record_node(rec_n, rec_b, r_g, r_aux, __builtin_amdgcn_readlane(ts, l), KA(rec_list), KA(rec_aux),
                            KA(tg_live), KA(tg_filt_tol), KA(ex_tcode), KA(hcnt_ex), (size_t)E, ei, KA(tg_cnt),
                            KA(tg_reg));
              bytes += 16 * (uint64_t)rec_n;
            }
            ex_pl = ei;
            break;
          }
        }
        if (FX_DIAG && lane == 0) g_sdiag[ex_bail ? 5 : ex_pl >= 0 ? 2 : 4] += 1;
        if (ex_bail) {  // a long scan: the full path's (nothing was placed; the failure memos stay valid)
          handoff = pod;
          fb = FB_SCAN;
          break;
        }
        // cursor: every position before the winner failed; with owned groups, before the first position that passed
        // the count-independent checks (a zone-count failure may pass later), as the full path
        const int cpos = TOPO && t_n ? min(ex_ipos, E) : (ex_pl >= 0 ? ex_pl : E);
        *reinterpret_cast<int2*>(&KA(cur_ex)[2 * sl]) = make_int2(cpos, a_cex_prev_stamp);  // (every lane)
        a_cex_prev_pos = cpos;
        if (ex_pl >= 0) {
          int ex_n = U(s_ctl[14]), ex_lost = U(s_ctl[21]);
          mstack_push_reg((int32_t LDS*)s_stk[1], ex_n, ex_lost, a_cex_prev_stamp + 1, ex_pl);
          {  // (uniform values: every lane stores, no exec-masked block)
            s_ctl[14] = ex_n;
            s_ctl[21] = ex_lost;
            s_ctl[15] = a_cex_prev_stamp + 1;
          }
          wave_sync();
          // the in-flight cursor is untouched (no in-flight scan): the next pod of this level reads the same one
          a_cur_prev_pos = cur;
          a_cur_prev_stamp = stamp;
          cont_w = -1;
          pops++;
          if (lane == n_buf) {
            buf_pod = pod;
            buf_pl = -2 - ex_pl;
          }
          if (++n_buf == 64) {
            KA(placement)[buf_pod] = buf_pl;
            KA(events)[n_ev + lane] = buf_pod;
            n_ev += 64;
            n_buf = 0;
          }
          FTF(13);  // diagnostic: FT(0) to an existing-node placement
          continue;
        }
      } else if (FL_HAS_EX) {  // addToExistingNode: every position fails (cursor == n_existing)
        if (FX_DIAG && lane == 0) g_sdiag[3] += 1;
        *reinterpret_cast<int2*>(&KA(cur_ex)[2 * sl]) = make_int2(KA(n_existing), a_cex_prev_stamp);  // (every lane)
        a_cex_prev_pos = KA(n_existing);
      }
      FT(1);
      // sort.Slice(newNodeClaims) replay + first-fit start (sort arrays in LDS or chunked; the flat global order:
      // the full path)
      if (UNLIKELY(!CHK && !in_lds)) {
        handoff = pod;
        fb = FB_SPILLED;
        break;
      }
      const LdsI32 ord = (LdsI32)s_dyn;
      const LdsI32 npods = (LdsI32)(s_dyn + KA(sort_cap));
      const ChkDir cd = chk_dir(s_dyn);
      const int c19 = (FL_SKIP & 2) ? cur : min(cur, mstack_query_wave((LdsI32)s_stk[0], stk_n, stk_lost, stamp));
      const int n_nc = n_nc_all;
      FTF(8);
      int low;
      bool n_moved = false;  // the pending mutation moved its NodeClaim (sort_mut1_window)
      const bool mut_was1 = mut == 1 && mut_p == cont_w;  // ... and it is the previous pod's commit at cont_w
      if (CHK) {
        low = mut == 0 ? -1 : chk_sort(cd, (ChkCtl LDS*)&g_chk, KA(chk_blk), n_nc, mut, mut_p, KA(g_order), KA(g_npods),
                                       &KA(stats)[31], h_ck, h_blk, h_id, h_key);
        h_ck = -1;  // (the replay may have moved entries)
        if (low == -4) {  // the literal pdqsort ran and its rebuild did not fit: the flat order, the full path's
          if (lane == 0) s_ctl[5] = 0;
          mut = 0;
          mstack_push_reg((int32_t LDS*)s_stk[0], stk_n, stk_lost, ++stk_t, 0);
        }
        if (low <= -3) {  // -3: nothing changed, the full path converts to the flat order and replays there
          handoff = pod;
          fb = FB_SHIFT;
          break;
        }
      } else {
        low = mut == 0 ? -1 : (mut == 1 ? ((FL_SKIP & 1) ? mut_p : sort_mut1_window(ord, npods, n_nc, mut_p, KA(sort_cap), &n_moved)) : -2);
        if (UNLIKELY(low == -2)) low = sort_newnodeclaims_wave(ord, npods, n_nc, mut, mut_p, 256, &KA(stats)[31]);
        if (UNLIKELY(low == -2)) {  // a long shift: the full path sorts (the pending mutation is still in s_ctl[10..11])
          handoff = pod;
          fb = FB_SHIFT;
          break;
        }
      }
      FTF(9);
      const int start = min(min(c19, low >= 0 ? low : INT32_MAX), n_nc);
      mut = 0;
      if (low >= 0 && !(FL_SKIP & 2)) mstack_push_reg((int32_t LDS*)s_stk[0], stk_n, stk_lost, ++stk_t, low);
      wave_sync();
      FT(2);
      if (memo) {  // the full path's failure: cursors at the end, Preferences.Relax, Queue.Push
        if (FX_DIAG && lane == 0) {  // diagnostic (config 5 has no existing nodes: the slots are free there)
          g_sdiag[0] += 1;
          if (cont_w >= 0) g_sdiag[2] += 1;
        }
        a_cur_prev_pos = n_nc;
        a_cur_prev_stamp = stk_t;
        const int lvl = sl - KA(shape_level_base)[shape];
        const bool relaxed = lvl + 1 < KA(shape_nlevels)[shape];
        int tail = q_head + q_len;
        if (tail >= KA(n_pods)) tail -= KA(n_pods);
        q_len += 1;
        {  // (uniform values: every lane stores, no exec-masked block)
          *reinterpret_cast<int2*>(&KA(cur_nc)[2 * sl]) = make_int2(n_nc, stk_t);
          KA(placement)[pod] = -1;
          if (relaxed) KA(pod_level)[pod] = lvl + 1;
          KA(queue)[tail] = pod;
          if (!relaxed) {
            KA(lastlen)[pod] = q_len;
            KA(lastlen_epoch)[pod] = epoch;
          }
        }
        if (relaxed) epoch += 1;  // lastLen = map{}
        memo_pops++;
        cont_w = -1;
        if (!relaxed && off + 1 < qw_n) {
          // the window entries right behind this pod that fail by the memo as well, at their last relaxation level:
          // their pops change nothing the next of them reads (no NodeClaim, mutation or relaxation, the queue length
          // stays len, the order stays as replayed), so each does exactly this pod's bookkeeping — cursors at the
          // end, placement -1, Queue.Push with lastLen = len — and they are done at once, window entry i on lane i,
          // up to the first that would end the Solve (popped again at the same length), needs the full path, or
          // breaks the run
          const int j0 = off + 1;
          const bool inw = lane >= j0 && lane < qw_n;
          const int gsl = inw ? qw_sl : 0, gsh = inw ? qw_shape : 0;  // (reads at valid indices, masked after)
          const int32_t sf = KA(sl_fail)[gsl];
          const int lb = KA(shape_level_base)[gsh], nl = KA(shape_nlevels)[gsh];
          const uint64_t hpc = KA(hp_any) ? KA(shape_hp_conf)[gsh] : 0;
          const bool ok = inw && sf == n_nc && gsl - lb + 1 >= nl && hpc == 0 &&
                          !(qw_epoch == epoch && qw_lastlen == q_len);
          const uint64_t okm = __ballot(ok) >> j0;
          const int k = min(__builtin_ctzll(~okm), pop_left - (pops + memo_pops));
          if (k > 0) {
            if (lane >= j0 && lane < j0 + k) {
              const int np = KA(n_pods);
              const int tail_i = (int)(((int64_t)q_head + q_len + (lane - j0)) % np);
              KA(placement)[qw_pod] = -1;
              KA(queue)[tail_i] = qw_pod;
              KA(lastlen)[qw_pod] = q_len;
              KA(lastlen_epoch)[qw_pod] = epoch;
              *reinterpret_cast<int2*>(&KA(cur_nc)[2 * gsl]) = make_int2(n_nc, stk_t);
              if (FL_HAS_EX) *reinterpret_cast<int2*>(&KA(cur_ex)[2 * gsl]) = make_int2(KA(n_existing), a_cex_prev_stamp);
            }
            q_head = (int)(((int64_t)q_head + k) % KA(n_pods));
            memo_pops += k;
            if (FX_DIAG && lane == 0) {
              g_sdiag[1] += k;
              g_sdiag[3] += 1;
            }
            qw_next = j0 + k;
            pf_off = -1;  // (the prefetched stage was the next entry's)
            prev_sl = -1;
          }
        }
        continue;
      }
      // addToInflightNode: pre-checks 64 positions at a time, then the append-path attempts in order. A long scan
      // is the full path's (512-lane pre-pass).
      int placed = -1, wpos = -1, why = FB_NONE, ipos = INT32_MAX;  // ipos: first count-independent pass (topology)
      // continuation: the previous pod (same shape-level) appended to NodeClaim c_nc at position cont_w, the replay
      // left it there, and the first-fit scan starts there (every earlier position failed this level and is
      // unchanged): the first candidate is c_nc itself, whose pre-check record, remaining types, requests and
      // threshold indices the wave holds from that commit — no gathers for this round (c_nc is tagged with the
      // level: memo NC_MERGED). A failed attempt falls back to the scan from the next position.
      bool cont = CONT && FAST_CONT && !CHK && !TOPO && c_nc >= 0 && cont_w >= 0 && cont_w == start &&
                  mut_was1 && !n_moved && sl == cont_sl && rr_b4p == 0 && c_hm == 0;
      bool bail = !CHK && n_nc - start > FAST_SCAN_MAX && !cont;
      if (bail) why = FB_SCAN;
      if (!(FL_SKIP & 4) && !bail) starts += (uint32_t)start;
      // chunked order: the start position's chunk and slot, the window of chunks whose live mask is in lm
      int ch0 = 0, cs0 = 0, cc = 0, lm_base = 0, n_live = 0;
      uint64_t lm = 0;
      const bool can_dead = CHK && !t_n && sl < KA(chk_dead_rows);
      int32_t* const deadrow = KA(chk_dead) + (size_t)(can_dead ? sl : 0) * CHK_MAXC;
      const int nch = CHK ? U(g_chk.nch) : 0;
      if (CHK) {
        ch0 = start < n_nc ? chk_find(cd, nch, start) : nch;
        cs0 = ch0 < nch ? start - cd.start[ch0] : 0;
        cc = ch0;
      }
      for (int base = start; placed == -1 && !bail;) {
        int i, ck = -1, nscan;  // position of this lane's entry; its chunk; entries this round scans
        bool valid;
        int nc, c_bid = 0, c_bkey = 0;
        if (CHK) {
          while (!lm && cc < nch) {  // the next window's live chunks (dead ones: every NodeClaim fails permanently)
            // (unconditional reads at a clamped directory index, masked after)
            const int b = ci_blk(cd.info[min(cc + lane, CHK_MAXC - 1)]);
            const bool dead = can_dead && deadrow[b] == cd.bep[b];
            const bool live = cc + lane < nch && !dead;
            lm = __ballot(live);
            lm_base = cc;
            cc = min(cc + 64, nch);
          }
          if (!lm) break;
          if (++n_live > FAST_CHK_LIVE) {  // a long scan: the full path's (4 chunks per round)
            bail = true;
            why = FB_SCAN;
            break;
          }
          ck = lm_base + __builtin_ctzll(lm);
          lm &= lm - 1;
          const uint32_t v = cd.info[ck];
          valid = lane < ci_cnt(v) && !(ck == ch0 && lane < cs0);
          // the chunk's block (ids and keys) in one batch: the winner's chunk is the next replay's
          const int bid_r = KA(chk_blk)[ci_blk(v)].id[lane], bkey_r = KA(chk_blk)[ci_blk(v)].key[lane];
          c_bid = lane < ci_cnt(v) ? bid_r : -1;
          c_bkey = lane < ci_cnt(v) ? bkey_r : INT32_MAX;
          nc = valid ? c_bid : 0;
          i = cd.start[ck] + lane;
          nscan = __popcll(__ballot(valid));
        } else if (cont) {  // the continuation round: position start alone, from registers
          if (base >= n_nc) break;
          i = base + lane;
          valid = lane == 0;
          nc = valid ? c_nc : 0;
          nscan = 1;
          base += 1;
        } else {
          if (base >= n_nc) break;
          if (n_nc - base > FAST_SCAN_MAX && base != start) {  // (after a failed continuation round: a long scan)
            bail = true;
            why = FB_SCAN;
            break;
          }
          i = base + lane;
          valid = i < n_nc;
          const int nc_r = ord[min(i, KA(sort_cap) - 1)];  // (unconditional read, masked after)
          nc = valid ? nc_r : 0;
          nscan = min(64, n_nc - base);
          base += 64;
        }
        const bool cont_round = !CHK && cont;
        cont = false;
        bool cand = false, tag = false, icand = false, pfail = false;
        int32_t ver = 0;
        HeadView hv{0, 0, 0, 0, 0, 0};
        // speculative loads of the first position's NodeClaim (the usual winner), issued ahead of the pre-check
        // gathers (and outside their lane-divergent block) so that the two round trips overlap
        const int nc0 = __builtin_amdgcn_readlane(nc, 0);
        uint64_t hm0 = c_hm, X00 = c_X;
        int cat0 = c_cat;
        int64_t rq0 = c_q;
        int32_t j00 = c_fj;
        if (nc0 != c_nc) {
          const KReqs* cr0 = kreq_at(KA(nc_reqs), nc0);
          hm0 = cr0->hmin & cr0->present;
          cat0 = KA(nc_cat)[nc0];
          // (unconditional reads at clamped lanes, masked after)
          const uint64_t x_r = KA(nc_X)[(size_t)nc0 * D.TW + min(lane, D.TW - 1)];
          const int64_t q_r = KA(nc_requests)[(size_t)nc0 * KP_NRES + min(lane, KP_NRES - 1)];
          const int32_t j_r = KA(nc_fitj)[(size_t)nc0 * KP_NRES + min(lane, KP_NRES - 1)];
          X00 = lane < D.TW ? x_r : 0;
          rq0 = lane < KP_NRES ? q_r : 0;
          j00 = lane < KP_NRES ? j_r : 0;
        }
        {
          // every gather issued unconditionally (the lanes past the order read NodeClaim 0 and are masked after): one
          // round trip and no exec-masked block
          int32_t fl = NC_MERGED;
          if (LIKELY(!cont_round)) {
            const int ncc_ = KA(ncc);
            const int32_t fl_r = KA(nc_fail)[(size_t)sl * ncc_ + min(nc, ncc_ - 1)];
            fl = nc < ncc_ ? fl_r : -2;
            const HeadView ld = load_head(KA(nc_head) + nc, four);
            const bool mine = nc == c_nc;
            hv = HeadView{mine ? c_r0 : ld.r0, mine ? c_r1 : ld.r1, mine ? c_r2 : ld.r2,
                          mine ? c_r3 : ld.r3, mine ? c_ver : ld.ver, mine ? c_ts : ld.ts};
          } else {
            hv = HeadView{c_r0, c_r1, c_r2, c_r3, c_ver, c_ts};
          }
          ver = hv.ver;
          const int32_t ts = hv.ts;
          bool fit = (hv.r0 >= pr0) & (hv.r1 >= pr1) & (hv.r2 >= pr2) & (hv.r3 >= pr3);
          if (UNLIKELY(rr_b4p)) {  // a fifth requested resource and beyond (that the pod requests)
            const int64_t* rq = KA(nc_requests) + (size_t)nc * KP_NRES;
            const int64_t* mx = KA(nc_maxalloc) + (size_t)nc * KP_NRES;
            for (uint32_t rm = rr_b4p; rm; rm &= rm - 1) {
              const int r = __builtin_ctz(rm);
              fit = fit & (rq[r] + lane_bcast_i64(preq_lane, r) <= mx[r]);
            }
          }
          cand = valid & fit & (fl != ver) & (fl != NC_NEVER) & (((tolmask >> ts) & 1) != 0);
          if (CHK) pfail = !fit || fl == NC_NEVER || !((tolmask >> ts) & 1);  // permanent (see the full path)
          bool pinned = true;  // every dictionary key the pod spreads over is one value on the NodeClaim
          if (TOPO && t_n) {
#pragma unroll
            for (int j = 0; j < 4; j++)
              if (j < t_n && t_key[j] < 0)
                cand = cand & ((int)KA(hcnt_nc)[(size_t)t_row[j] * KA(hnc_stride) + nc] + t_self[j] <= t_mskew[j]);
            icand = cand;
#pragma unroll
            for (int j = 0; j < 4; j++)
              if (j < t_n && t_key[j] >= 0) {
                const uint32_t code = KA(nc_tcode)[(size_t)t_slot[j] * KA(hnc_stride) + nc];
                cand = cand & ((code == 0xFF) | ((code < 64) & (((t_acc[j] >> (code & 63)) & 1) != 0)));
                pinned = pinned && code < 64;
              }
          }
          tag = cand && (fl >= NC_MERGED || triv) && pinned;
        }
        if (!(FL_SKIP & 4)) n_scan += (uint32_t)nscan;
        uint64_t cm = __ballot(cand);
        const uint64_t tm = __ballot(tag);
        if (TOPO && t_n && ipos == INT32_MAX) {
          const uint64_t im = __ballot(icand);
          if (im) ipos = __builtin_amdgcn_readlane(i, __builtin_ctzll(im));
        }
        if (can_dead && !(ck == ch0 && cs0 > 0) && __ballot(valid && !pfail) == 0) {  // (uniform: every lane)
          const int b = ci_blk(cd.info[ck]);  // every NodeClaim of the chunk fails the shape-level permanently
          deadrow[b] = cd.bep[b];
        }
        // the next pod's prefetch was issued before these gathers, so it has landed: take it off the outstanding
        // list now rather than at the next pod's stage, where the wait would cover this pod's stores as well
        READY(pf_own);
        if (TOPO) READY(pf_stg);
        READY(pf_ce0);
        READY(pf_ce1);
        READY(pf_preq);
        READY(pf_tol);
        READY(pf_cur);
        READY(pf_stamp);
        FT(3);
        while (cm) {
          const int l = __builtin_ctzll(cm);
          cm &= cm - 1;
          const bool tagged = (tm >> l) & 1;  // the NodeClaim already carries this shape-level (append path)
          const int ncx = __builtin_amdgcn_readlane(nc, l);
          const int32_t verx = __builtin_amdgcn_readlane(ver, l);  // NodeClaim's version (no reload after stores)
          attempts++;
          uint64_t hm = hm0, X0 = X00;
          int cat = cat0;
          int64_t rq_lane = rq0;
          int32_t j0_lane = j00;
          if (l != 0 && ncx == c_nc) {
            hm = c_hm, X0 = c_X, cat = c_cat, rq_lane = c_q, j0_lane = c_fj;
          } else if (l != 0) {
            const KReqs* cr = kreq_at(KA(nc_reqs), ncx);
            hm = cr->hmin & cr->present;
            cat = KA(nc_cat)[ncx];
            const uint64_t x_r = KA(nc_X)[(size_t)ncx * D.TW + min(lane, D.TW - 1)];
            const int64_t q_r = KA(nc_requests)[(size_t)ncx * KP_NRES + min(lane, KP_NRES - 1)];
            const int32_t j_r = KA(nc_fitj)[(size_t)ncx * KP_NRES + min(lane, KP_NRES - 1)];
            X0 = lane < D.TW ? x_r : 0;
            rq_lane = lane < KP_NRES ? q_r : 0;
            j0_lane = lane < KP_NRES ? j_r : 0;
          }
          FTF(10);
          const int64_t q_lane = rq_lane + preq_lane;
          // append path (merged before, no minValues): Fits over the remaining types; otherwise NodeClaim.Add in
          // full, as the full path's attempt: Compatible + Add of the requirements, then the type filter
          const bool full_add = !tagged || hm;
          if (TOPO && t_n && full_add) {  // the merge narrows by the counts (topo_narrow): the full path's
            why = FB_MERGE;
            bail = true;
            break;
          }
          uint64_t X = 0, m_v = 0;
          ReqView rv;
          bool perm = true;  // a failure here is permanent (NC_NEVER) unless it is Compatible's undefined-key rule
          if (LIKELY(!full_add)) {
            if (LIKELY(n_rrp <= 4 && cat < 8)) {
              X = fits_lean(D, (const CatHdr LDS*)&g_hdr[cat], X0, q_lane, j0_lane, (const int64_t LDS*)g_fitv, rrp,
                            n_rrp, fnb, (int32_t LDS*)fl_fitj);
            } else {
              X = fl_fits_filter(cat, X0, q_lane, j0_lane, KA(req_res_mask), (uint64_t)(uintptr_t)KA(cats));
              bytes += fl_io[1];
            }
            n_app++;
          } else {
            if (!b_staged) {  // the pod's requirement set, once per pod
              constexpr int NQ = (int)(sizeof(KReqs) / 8);
              const uint64_t* src = reinterpret_cast<const uint64_t*>(KA(shape_reqs) + (size_t)sl * sizeof(KReqs));
              uint64_t* dstB = reinterpret_cast<uint64_t*>(&fl_B);
              for (int i = lane; i < NQ; i += 64) dstB[i] = src[i];
              wave_sync();
              b_staged = true;
            }
            const CandReq crx = load_cand(D, kreq_at(KA(nc_reqs), ncx));
            const VInt vig = vint_global(KA(vint));
            const uint64_t b_negop = KA(shape_negop)[sl];
            bool mok = merge_compatible(D, crx, (const KReqs*)&fl_B, b_negop, true, m_v, rv,
                                        (WaveSlots*)&fl_slots, vig);
            if (!mok) perm = (fl_B.present & ~crx.P & ~b_negop & ~D.wellknown) == 0;
            bytes += sizeof(KReqs);
            if (mok) {
              const int pb = KA(pvp_base)[sl * KA(n_catalogs) + cat];
              const uint64_t* pvp = KA(shape_pvp) + (size_t)pb * D.TW;
              X = filter_types(D, hdr(cat), rv, m_v, X0, fl_B.present, pvp, KA(pvp_slot) + (size_t)sl * KP_MAX_KEYS,
                               q_lane, j0_lane, (const int64_t LDS*)g_fitv, KA(req_res_mask), vig, (uint32_t*)fl_scratch,
                               (RowPtr LDS*)fl_rl, &bytes, fl_fitj);
              bytes += (uint64_t)D.TW * 8 + KP_NRES * 8;
            }
          }
          FTF(11);
          if (LIKELY(__ballot(X != 0))) {
            // Topology.Record's reads ahead of the stores (a merge may set the NodeClaim's value codes: then the
            // code is read again after store_tcodes)
            RecRead rrd{0, 0, false};
            if (TOPO && rec_n && rec_n <= 64)
              rrd = record_read(rec_n, r_g, r_aux, __builtin_amdgcn_readlane(hv.ts, l), KA(tg_live), KA(tg_filt_tol),
                                KA(nc_tcode), KA(hcnt_nc), (size_t)KA(hnc_stride), ncx, KA(tg_reg));
            if (UNLIKELY(full_add)) {
              store_merged(reinterpret_cast<KReqs*>(KA(nc_reqs) + (size_t)ncx * sizeof(KReqs)), rv, m_v, D.W, D.KB);
              if (TOPO && KA(n_tk)) store_tcodes(KA(n_tk), KA(tk_keys), KA(nc_tcode), KA(hnc_stride), rv, m_v, ncx);
              if (ncx < KA(ncc)) KA(nc_fail)[(size_t)sl * KA(ncc) + ncx] = NC_MERGED;  // (uniform: every lane)
            }
            // the remaining types and threshold indices are stored only when they changed (the append path
            // usually leaves both as they were): fewer vector-memory operations ahead of the next pod's loads
            const int32_t fj_r = fl_fitj[min(lane, KP_NRES - 1)];  // (unconditional, masked after)
            const int32_t fj = lane < KP_NRES ? fj_r : 0;
            if (UNLIKELY(__ballot(lane < D.TW && X != X0))) {
              if (lane < D.TW) KA(nc_X)[(size_t)ncx * D.TW + lane] = X;
            }
            if (lane < KP_NRES) KA(nc_requests)[(size_t)ncx * KP_NRES + lane] = q_lane;
            if (UNLIKELY(__ballot(lane < KP_NRES && fj != j0_lane))) {
              if (lane < KP_NRES) KA(nc_fitj)[(size_t)ncx * KP_NRES + lane] = fj;
            }
            if (!CHK) {  // len(Pods) + 1: one uniform read, every lane writes the same value (no exec-masked block)
              const int cnt1 = npods[ncx] + 1;
              npods[ncx] = cnt1;
            }
            if (lane == 0) {
              if (CHK) {  // len(Pods) in the chunk's block (the replay reads it there) and the flat copy
                KA(chk_blk)[ci_blk(cd.info[ck])].key[l] += 1;
                KA(g_npods)[ncx] += 1;
              }
            }
            // the pre-check record, from lane l's copy: headroom minus the pod, version + 1 (kept lane-masked: the
            // broadcast for an all-lane store measured +0.5 % on config 2)
            if (lane == l) {
              int4* hp = reinterpret_cast<int4*>(KA(nc_head) + ncx);
              const int64_t n0 = hv.r0 - pr0, n1 = hv.r1 - pr1;
              hp[0] = make_int4((int)n0, (int)(n0 >> 32), (int)n1, (int)(n1 >> 32));
              if (four) {
                const int64_t n2 = hv.r2 - pr2, n3 = hv.r3 - pr3;
                hp[1] = make_int4((int)n2, (int)(n2 >> 32), (int)n3, (int)(n3 >> 32));
              }
              KA(nc_head)[ncx].ver = verx + 1;
            }
            placed = ncx;
            wpos = __builtin_amdgcn_readlane(i, l);
            if (CHK) {  // the block as the commit left it, for the next pod's replay
              h_ck = ck;
              h_blk = ci_blk(cd.info[ck]);
              h_id = c_bid;
              h_key = c_bkey + (lane == l ? 1 : 0);
            }
            if (TOPO && triv && ncx < KA(ncc)) KA(nc_fail)[(size_t)sl * KA(ncc) + ncx] = NC_MERGED;
            if (TOPO && rec_n) {
              // Topology.Record, as the full path's: each recorded group (spreads only on fast levels) on its own lane;
              // a dictionary key counts once the NodeClaim holds one value of it (its value code < 64)
              if (LIKELY(rec_n <= 64 && !full_add))
                record_write(rrd, r_g, r_aux, KA(hcnt_nc), (size_t)KA(hnc_stride), ncx, KA(tg_cnt), KA(tg_reg));
              else
                record_node(rec_n, rec_b, r_g, r_aux, __builtin_amdgcn_readlane(hv.ts, l), KA(rec_list), KA(rec_aux),
                            KA(tg_live), KA(tg_filt_tol), KA(nc_tcode), KA(hcnt_nc), (size_t)KA(hnc_stride), ncx,
                            KA(tg_cnt), KA(tg_reg));
              bytes += 16 * (uint64_t)rec_n;
            }
            if (LIKELY(!full_add)) {  // the append path left the requirements (hmin, catalogue) as they were
              c_nc = ncx, c_cat = cat, c_hm = hm, c_X = X, c_q = q_lane, c_fj = fj;
              c_r0 = lane_bcast_i64(hv.r0, l) - pr0;
              c_r1 = lane_bcast_i64(hv.r1, l) - pr1;
              c_r2 = four ? lane_bcast_i64(hv.r2, l) - pr2 : INT64_MAX;  // (load_head's value for unused slots)
              c_r3 = four ? lane_bcast_i64(hv.r3, l) - pr3 : INT64_MAX;
              c_ver = verx + 1, c_ts = __builtin_amdgcn_readlane(hv.ts, l);
            } else {
              c_nc = -1;
            }
            FTF(12);
            break;
          }
          if (ncx < KA(ncc)) KA(nc_fail)[(size_t)sl * KA(ncc) + ncx] = perm ? NC_NEVER : verx;  // (every lane)
        }
      }
      wave_sync();
      FT(4);
      if (UNLIKELY(placed == -1)) {  // templates, a merge, minValues or a long scan: the full path takes over this pod
        handoff = pod;
        fb = why;
        break;
      }
      pops++;
      cont_w = c_nc >= 0 ? wpos : -1;  // (c_nc: this commit was an append, its NodeClaim held in registers)
      cont_sl = sl;
      // cursor: every position before the winner failed; with owned groups, before the first position that passed
      // the count-independent checks (a zone-count failure may pass later), as the full path
      const int cpos = TOPO && t_n ? min(ipos, wpos) : wpos;
      a_cur_prev_pos = cpos;
      a_cur_prev_stamp = stk_t;
      mut = 1;
      mut_p = wpos;
      // (every lane stores the same 8 bytes: one coalesced store, no exec-masked block)
      *reinterpret_cast<int2*>(&KA(cur_nc)[2 * sl]) = make_int2(cpos, a_cur_prev_stamp);
      // placement / events: buffered one pod per lane, written 64 at a time (nothing reads them before the
      // fast lane returns)
      if (lane == n_buf) {
        buf_pod = pod;
        buf_pl = placed;
      }
      if (UNLIKELY(++n_buf == 64)) {
        KA(placement)[buf_pod] = buf_pl;
        KA(events)[n_ev + lane] = buf_pod;
        n_ev += 64;
        n_buf = 0;
      }
      // ---- run-length commit (the continuation variant: queue runs of one shape-level). The next k window entries
      // share this pod's level, and for each of them, one at a time, the reference would do exactly what it just did:
      // sort.Slice leaves this NodeClaim where it is (the entry after it keeps len(Pods) >= its own), the first-fit
      // scan starts at its position (every earlier one failed the level and is unchanged), and NodeClaim.Add is Fits
      // over its remaining types with every requested resource still under the threshold value it just passed (the
      // remaining types, and so the result, unchanged). k is the largest count for which all of that holds in
      // closed form; the k pods are committed at once: requests + k * pod, len(Pods) + k, headroom - k * pod, version
      // + k, the same cursor and one mutation-stack entry for the k identical ones. Anything else: the pod loop.
      if (CONT && cont_w == wpos && c_cat == 0 && c_hm == 0 && rr_b4p == 0 && n_rrp <= 4) {
        const int e = off + 1 + lane;  // lane j: the j-th window entry after this pod
        const int e_sl = __shfl(qw_sl, e & 63, 64), e_ep = __shfl(qw_epoch, e & 63, 64),
                  e_ll = __shfl(qw_lastlen, e & 63, 64), e_pod = __shfl(qw_pod, e & 63, 64);
        // Queue.Pop would stop at an entry last pushed at the length it would pop it at (lastLen)
        const bool ok = e < qw_n && e_sl == sl && !(e_ep == epoch && e_ll == q_len - lane);
        const uint64_t okm = __ballot(ok);
        int k = (int)__builtin_ctzll(~okm);
        // sort.Slice: batched pod m (1-based) replays len(Pods) = c + m - 1 at wpos against the next entry's
        const int c1 = npods[placed];
        const int nxt = wpos + 1 < n_nc_all ? npods[ord[wpos + 1]] : INT32_MAX;
        if (nxt != INT32_MAX) k = min(k, max(0, nxt - c1 + 1));
        // Fits: every requested resource stays at or under the threshold value of its current index
        int kf = INT32_MAX;
        if (lane < KP_NRES && preq_lane > 0) {
          const int slot = g_hdr[0].fit_slot[lane], n = g_hdr[0].fit_n[lane];
          kf = 0;
          if (slot >= 0 && c_fj < n) {
            const int64_t room = g_fitv[slot * FITV_CAP + c_fj] - c_q;
            kf = room >= 0 ? (int)min<int64_t>(room / preq_lane, 64) : 0;
          }
        }
        k = min(k, wave_min_i32(kf));
        k = min(k, 63);
        if (k > 0) {
          const int64_t kk = k;
          // the NodeClaim: requests, len(Pods), pre-check record (headroom, version)
          c_q += kk * preq_lane;
          {
            const int64_t q_top = lane_bcast_i64(c_q, KP_NRES - 1);
            KA(nc_requests)[(size_t)placed * KP_NRES + min(lane, KP_NRES - 1)] = lane < KP_NRES ? c_q : q_top;
          }
          c_r0 -= kk * pr0, c_r1 -= kk * pr1;
          if (four) c_r2 -= kk * pr2, c_r3 -= kk * pr3;
          c_ver += k;
          {  // (uniform values, every lane stores)
            npods[placed] = c1 + k;
            int4* hp = reinterpret_cast<int4*>(KA(nc_head) + placed);
            hp[0] = make_int4((int)c_r0, (int)(c_r0 >> 32), (int)c_r1, (int)(c_r1 >> 32));
            if (four) hp[1] = make_int4((int)c_r2, (int)(c_r2 >> 32), (int)c_r3, (int)(c_r3 >> 32));
            KA(nc_head)[placed].ver = c_ver;
          }
          // the k replays: one mutation-stack entry at wpos (k identical pushes leave just the last), the cursor
          stk_t += k;
          mstack_push_reg((int32_t LDS*)s_stk[0], stk_n, stk_lost, stk_t, wpos);
          a_cur_prev_stamp = stk_t;
          *reinterpret_cast<int2*>(&KA(cur_nc)[2 * sl]) = make_int2(wpos, stk_t);
          // the k pods: popped, placed (events in queue order after the buffered ones)
          if (n_buf + k > 64) {
            if (lane < n_buf) {
              KA(placement)[buf_pod] = buf_pl;
              KA(events)[n_ev + lane] = buf_pod;
            }
            n_ev += n_buf;
            n_buf = 0;
          }
          const int bp = __shfl(e_pod, (lane - n_buf) & 63, 64);
          if (lane >= n_buf && lane < n_buf + k) {
            buf_pod = bp;
            buf_pl = placed;
          }
          n_buf += k;
          if (n_buf == 64) {
            KA(placement)[buf_pod] = buf_pl;
            KA(events)[n_ev + lane] = buf_pod;
            n_ev += 64;
            n_buf = 0;
          }
          q_head += k;
          if (q_head >= KA(n_pods)) q_head -= KA(n_pods);
          q_len -= k;
          qw_next = off + 1 + k;
          pf_off = -1;
          pops += k;
          attempts += k;
          n_app += (uint32_t)k;
          n_scan += (uint32_t)k;
          n_run += (uint32_t)k;
        }
      }
      FT(5);
    }
    if (lane < n_buf) {
      KA(placement)[buf_pod] = buf_pl;
      KA(events)[n_ev + lane] = buf_pod;
    }
    n_ev += n_buf;
#undef FT
#undef FTF
#undef FL_HAS_EX
#undef KA
  
  // write back: control block, window, counters, hand-off
  if (lane == 0) {
    s_ctl[0] = q_head;
    s_ctl[1] = q_len;
    s_ctl[3] = epoch;
    s_ctl[4] = n_ev;
    s_ctl[10] = mut;
    s_ctl[11] = mut_p;
    s_ctl[12] = stk_n;
    s_ctl[13] = stk_t;
    s_ctl[20] = stk_lost;
    s_ctl[32] = chk_next;
    if (handoff >= 0) {
      s_ctl[6] = handoff;
      s_ctl[26] = 1;
    }
    S->qw_head = qw_head;
    S->qw_n = qw_n;
    S->qw_next = qw_next;
    bytes += (uint64_t)fnb.probes * 512 + (uint64_t)fnb.rows * D.TW * 8 + (uint64_t)fnb.lb8 * 8 +
             (uint64_t)n_app * ((uint64_t)D.TW * 8 + KP_NRES * 8 + 8) + (uint64_t)n_scan * (12 + 16 * A->n_req_res);
    S->bytes += bytes;
    S->attempts += attempts;
    S->scanned += n_scan;
    S->starts += starts;
    S->fpods += pops;
    S->runpods += n_run;
    for (int i = 0; i < 14; i++) S->fcyc[i] += fcyc[i];
    if (fb >= 0) S->fbail[fb] += 1;
    S->fbail[FB_MEMO] += memo_pops;  // (not a hand-off: the pods the lane failed by the memo)
  }
  S->qw_pod[lane] = qw_pod;
  S->qw_shape[lane] = qw_shape;
  S->qw_sl[lane] = qw_sl;
  S->qw_lastlen[lane] = qw_lastlen;
  S->qw_epoch[lane] = qw_epoch;
  wave_sync();
  return pops + memo_pops;
}

// TOPO: the batch has topology spread groups (else that code compiles out). BATCH: one Solve per workgroup, each with
// its own arguments batch[blockIdx.x] (the general consolidation path's simulations); else the kernel argument a0.
#if KP_TU & 1
template <int NW, bool TOPO, bool BATCH>
__global__ __launch_bounds__(NW * 64) void solve_kernel(SolveArgs a0, const SolveArgs* __restrict__ batch) {
  const SolveArgs& a = BATCH ? batch[blockIdx.x] : a0;
  constexpr int NT = NW * 64;
  DevDict& D = g_D;
  __shared__ WaveSlots slots[NW];
  __shared__ int32_t s_ok[NW];
  __shared__ int32_t s_wcnt[4 * NW];
  int32_t (&s_ctl)[34] = g_ctl;
  auto& s_stk = g_stk;  // mutation stacks: [0] in-flight positions, [1] existing positions
  __shared__ int32_t s_list[4 * NT];
  __shared__ uint32_t s_scratch[NW][2 * KP_MAX_WORDS];
  __shared__ KReqs s_B;  // the popped pod's requirements, staged once per pod
  __shared__ int32_t s_fitj[NW][KP_NRES];
  __shared__ int64_t s_preq[KP_NRES];          // pod requests (staged per pod)
  __shared__ int32_t s_pslot[KP_MAX_KEYS];     // PVP row of each pod key (staged per pod)
  auto& s_fitv = g_fitv;  // Fits threshold values of catalogue 0 (CatHdr.fit_slot rows)
  __shared__ TopoOwn s_town[8];                 // owned topology groups of the popped pod (staged per pod)
  __shared__ uint64_t s_tacc[8];
  __shared__ int32_t s_tcnt[8][64];
  __shared__ uint64_t s_tsub[8];  // KP_TIMING: wave 0's attempt split (merge, pod-key rows, Fits rows, row loads, minValues, n)
  __shared__ int64_t s_vint[KP_MAX_BOUND_KEYS * 64];  // parsed integers of the bounded keys' first value words
  __shared__ RowPtr s_rl[NW][RL_CAP];                 // per-wave row lists (filter_types)
  __shared__ int32_t s_pvpb[32];                      // PVP row base of the popped pod per catalogue (staged per pod)
  auto& s_hdr = g_hdr;  // catalogue descriptors 0..7
  __shared__ CatHdr s_hdrw[NW];                       // per-wave descriptor of a catalogue >= 8
  extern __shared__ int32_t s_dyn[];  // ord[a.sort_cap], npods[a.sort_cap] while n_nc <= a.sort_cap
  __shared__ int32_t s_rcap[KP_MAX_CLASSES];  // remaining capacity per reservation class (ReservationManager)
  __shared__ uint64_t s_topo_keys;            // the popped pod's spread keys (staged per pod)

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = LANE;
  block_copy(D, a.dict);
  __syncthreads();
  for (int i = tid; i < D.KB * 64; i += NT) s_vint[i] = a.vint[i];
  if (tid < KP_MAX_CLASSES) s_rcap[tid] = a.res_cap0[tid];
  const bool res_strict = a.res_mode == 2;
  const int ncat_lds = min(a.n_catalogs, 8);
  for (int c = wave; c < ncat_lds; c += NW) hdr_fill_wave((CatHdr LDS*)&s_hdr[c], &a.cats[c], D.C);
  __syncthreads();
  // catalogue c's descriptor in LDS: catalogues >= 8 are copied into the wave's slot first (one round trip)
  auto hdr = [&](int c) -> const CatHdr LDS* {
    if (c < 8) return (const CatHdr LDS*)&s_hdr[c];
    hdr_fill_wave((CatHdr LDS*)&s_hdrw[wave], &a.cats[c], D.C);
    wave_sync();
    return (const CatHdr LDS*)&s_hdrw[wave];
  };
  const VInt vi{(const int64_t LDS*)s_vint, a.vint, D.KB};
  // the (first two) requested resources, whose pre-pass bounds are gathered unconditionally; the rest lazily.
  // With fewer than two, the slot repeats resource 0/1 (an unrequested resource: 0 + 0 <= value, vacuous only
  // if that value is >= 0, so such slots point at a requested one when there is one)
  const uint32_t rmask_all = a.req_res_mask;
  const int rr0 = rmask_all ? __builtin_ctz(rmask_all) : 0;
  const uint32_t rm1 = rmask_all & (rmask_all - 1);
  const int rr1 = rm1 ? __builtin_ctz(rm1) : rr0;
  const uint32_t rr_rest = rm1 & (rm1 - 1);
  const int rk2 = kth_res(rmask_all, 2), rk3 = kth_res(rmask_all, 3);  // pre-check record: resources 0..3
  uint32_t rr_b4 = rr_rest;
  for (int i = 0; i < 2 && rr_b4; i++) rr_b4 &= rr_b4 - 1;
  const bool four = rk2 >= 0;
  {  // Fits threshold tables of catalogue 0 for the first FITV_RES requested resources -> LDS
    int slot = 0;
    for (int r = 0; r < KP_NRES; r++) {
      const int64_t* g = s_hdr[0].d.fit_vals + (size_t)r * D.T;
      const int n = s_hdr[0].fit_n[r];
      const bool stage = ((a.req_res_mask >> r) & 1) && slot < FITV_RES && n <= FITV_CAP;
      if (stage) {
        for (int i = tid; i < n; i += NT) s_fitv[slot * FITV_CAP + i] = g[i];
        if (tid == 0) s_hdr[0].fit_slot[r] = slot;
        slot++;
      }
    }
  }
  __syncthreads();
  uint64_t bytes = 0, attempts = 0, pops = 0, scanned = 0, starts = 0;
  const uint64_t pop_cap = (uint64_t)a.n_pods * 64 + 65536;  // Queue.Pop bound for the runaway guard
  int fl_fail = 0, fl_skip = 0;  // fast-lane backoff (wave 0)
  uint64_t tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
  const bool timing = a.timing && tid == 0;
  if (tid < 8) s_tsub[tid] = 0;
#define TS(ph)                                          \
  if (timing) {                                         \
    const uint64_t tnow = __builtin_amdgcn_s_memtime(); \
    tph[ph] += tnow - tlast;                            \
    tlast = tnow;                                       \
  }
  if (timing) tlast = __builtin_amdgcn_s_memtime();
  // control block (thread 0 owns): 0 head, 1 len, 2 n_nc, 3 lastLen epoch, 4 n_events, 5 order mode (1 sort arrays in
  // LDS, 2 chunked, 0 flat global), 6 pod
  if (tid == 0) {
    s_ctl[0] = 0;
    s_ctl[1] = a.n_pods;
    s_ctl[2] = 0;
    s_ctl[3] = 1;
    s_ctl[4] = 0;
    s_ctl[5] = 1;
    g_chk.nch = g_chk.nfree = g_chk.epoch = 0;
    g_chk.maxc = min(a.chk_maxc, CHK_MAXC);
    g_chk.nch_peak = g_chk.splits = g_chk.removals = g_chk.rebuilds = 0;
    s_ctl[10] = 0;  // pending mutation of newNodeClaims since the last sort: 0 none, 1 +1 at s_ctl[11], 2 appended
    s_ctl[11] = 0;
    s_ctl[12] = 0;  // in-flight mutation stack size / time / lost
    s_ctl[13] = 0;
    s_ctl[20] = -1;
    s_ctl[14] = 0;  // existing-node mutation stack size / time / lost
    s_ctl[15] = 0;
    s_ctl[21] = -1;
    s_ctl[17] = 0;  // existing scan start for the popped pod
    s_ctl[22] = 0;  // in-flight cursor of the popped pod's shape-level (staged)
    s_ctl[23] = 0;
    s_ctl[26] = 0;  // 1: the fast lane popped s_ctl[6] and hands it to the full path
    s_ctl[32] = 0;  // kp_cancel: pops at which the flag is read next; [33] 1: the Solve was cancelled
    s_ctl[33] = 0;
    g_fast.qw_head = 0;  // the fast lane's Queue window (empty) and counters
    g_fast.qw_n = 0;
    g_fast.qw_next = -1;
    g_fast.bytes = g_fast.attempts = g_fast.scanned = g_fast.starts = g_fast.fpods = g_fast.runpods = 0;
    for (int i = 0; i < 16; i++) g_fast.fcyc[i] = 0;
    for (int i = 0; i < 8; i++) g_fast.fbail[i] = 0;
    if (SORT_DIAG || EX_DIAG || FX_DIAG)
      for (int i = 0; i < 6; i++) g_sdiag[i] = 0;
  }
  __syncthreads();

  for (;;) {
    // a consolidation simulation (general path) whose Solve has made stop_nc (2) NodeClaims: computeConsolidation's
    // decision is already a no-op ("len(NewNodeClaims) != 1"; NodeClaims are never removed), so the rest of the Solve
    // cannot change it (uniform: s_ctl[2] was written before the previous iteration's barrier)
    if (BATCH && a.stop_nc > 0 && s_ctl[2] >= a.stop_nc) break;
    // ---- fast lane: wave 0 alone places every pod whose placement needs no requirement merge ----------------
    // The pod owns/feeds no topology group, every existing node is known to fail it (first-fit cursor), and the
    // first in-flight NodeClaim (sort order) that passes the pre-checks already carries the pod's shape-level
    // (NC_MERGED) without minValues: NodeClaim.Add is then Fits over the remaining types, evaluated in order
    // until one succeeds. The steps, decisions and state writes are the full path's (below), done by one wave
    // without workgroup barriers. Any other situation hands the popped pod to the full path (s_ctl[26]).
    if (FASTLANE && wave == 0 && !a.res_mode) {  // (reservation accounting runs on the full path only)
      // the call costs a few thousand cycles (register saves): after calls that placed nothing (topology-owning
      // or unschedulable pods), skip it for a growing number of pops; results do not depend on which path places
      if (fl_skip > 0) {
        fl_skip--;
      } else {
        // the Solve's argument block: the kernarg segment (a0 is the first argument), or its entry of the batch
        const uint64_t kargs = BATCH ? (uint64_t)&batch[blockIdx.x] : (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
        // instantiations: chunked order or not, existing nodes or none (compiled out), the continuation round (LDS
        // order, no topology, queue runs of one shape)
        int placed_fast;
        if (s_ctl[5] == 2)
          placed_fast = a.n_existing ? fast_lane<TOPO, true, true, false>(kargs, (int32_t LDS*)s_dyn, pops)
                                     : fast_lane<TOPO, true, false, false>(kargs, (int32_t LDS*)s_dyn, pops);
        else if (a.n_existing)
          placed_fast = fast_lane<TOPO, false, true, false>(kargs, (int32_t LDS*)s_dyn, pops);
        else if (!TOPO && a.cont)
          placed_fast = fast_lane<TOPO, false, false, !TOPO>(kargs, (int32_t LDS*)s_dyn, pops);
        else
          placed_fast = fast_lane<TOPO, false, false, false>(kargs, (int32_t LDS*)s_dyn, pops);
        pops += placed_fast;
        fl_fail = placed_fast ? 0 : fl_fail + 1;
        fl_skip = fl_fail >= 2 ? min(1 << min(fl_fail - 2, 6), 64) : 0;
      }
    }
    __syncthreads();
    // ---- Queue.Pop: stop when the head pod was last pushed at the current queue length ----------
    if (tid == 0) {
      const int len = s_ctl[1];
      int pod = -1;
      if (a.cancel && !s_ctl[33] && (int)pops >= s_ctl[32]) {  // ctx.Done(): the flag, at most every 1024 pops
        s_ctl[32] = (int)pops + 1024;
        if (cancel_set(a.cancel)) s_ctl[33] = 1;
      }
      if (pops > pop_cap) {  // runaway guard (a correct Solve stays far below): end the launch, report it
        a.stats[7] = 1;
      } else if (s_ctl[33]) {  // cancelled: end the launch without placing the rest (the host reports KP_E_CANCELED)
        a.stats[46] = 1;
      } else if (s_ctl[26]) {  // popped by the fast lane
        pod = s_ctl[6];
        s_ctl[26] = 0;
      } else if (len > 0) {
        const int head = s_ctl[0];
        const int p = a.queue[head];
        if (!(a.lastlen_epoch[p] == s_ctl[3] && a.lastlen[p] == len)) {
          pod = p;
          s_ctl[0] = head + 1 == a.n_pods ? 0 : head + 1;
          s_ctl[1] = len - 1;
        }
      }
      s_ctl[6] = pod;
    }
    __syncthreads();
    const int pod = s_ctl[6];
    if (pod < 0) break;
    pops++;
    const int shape = a.pod_shape[pod];
    const int lvl = a.pod_level[pod];
    const int sl = a.shape_level_base[shape] + lvl;
    {
      const uint64_t* src = reinterpret_cast<const uint64_t*>(kreq_at(a.shape_reqs, sl));
      uint64_t* dst = reinterpret_cast<uint64_t*>(&s_B);
      for (int i = tid; i < (int)(sizeof(KReqs) / 8); i += NT) dst[i] = src[i];
      if (tid < KP_NRES) s_preq[tid] = a.shape_requests[(size_t)shape * KP_NRES + tid];
      else if (tid >= 64 && tid < 64 + KP_MAX_KEYS) s_pslot[tid - 64] = a.pvp_slot[(size_t)sl * KP_MAX_KEYS + tid - 64];
      else if (tid >= 192 && tid < 192 + 32 && tid - 192 < a.n_catalogs)
        s_pvpb[tid - 192] = a.pvp_base[sl * a.n_catalogs + tid - 192];
      else if (tid == 128) {  // first-fit cursors of the shape-level (LDS stacks: no global round trips)
        const int ce = a.n_existing ? min(a.cur_ex[2 * sl], mstack_query((LdsI32)s_stk[1], s_ctl[14], s_ctl[21], a.cur_ex[2 * sl + 1])) : 0;
        s_ctl[17] = min(ce, a.n_existing);
        s_ctl[22] = a.cur_nc[2 * sl];
        s_ctl[23] = a.cur_nc[2 * sl + 1];
        s_ctl[24] = INT32_MAX;  // first count-independent pass (existing / in-flight), topology shape-levels
        s_ctl[25] = INT32_MAX;
        s_ctl[27] = 0;  // addToNewNodeClaim met a ReservedOfferingError
        // the unschedulable memo (SolveArgs::sl_fail): no NodeClaim created since a pod of this level failed everything
        s_ctl[31] = !TOPO && !a.res_mode && a.sl_fail[sl] == s_ctl[2];
        if (TOPO) {  // the shape-level's owned groups (count, base) and spread keys, staged with the cursors
          const int on = a.sl_own_n[sl];
          s_ctl[28] = on;
          s_ctl[29] = a.sl_own_base[sl];
          s_topo_keys = on ? a.sl_topo_keys[sl] : 0;
        }
      }
    }
    __syncthreads();
    TS(0);
    const uint64_t exdS = EX_DIAG ? __builtin_amdgcn_s_memtime() : 0;
    const KReqs* B = &s_B;
    const uint64_t b_negop = a.shape_negop[sl];
    const uint64_t tolmask = a.shape_tolerates[sl];
    const uint64_t hpc = a.hp_any ? a.shape_hp_conf[shape] : 0, hpa = a.hp_any ? a.shape_hp_add[shape] : 0;
    int placed = -1;  // >= 0 NodeClaim id; <= -2 existing node; -1 not placed
    // a memo hit fails the pod without the scans: the existing and in-flight cursors move to the end as a failed scan
    // leaves them, and the sort replay still runs (the order every later pod sees is the reference's)
    const bool memo_fail = s_ctl[31] != 0;
    // ---- topology: stage the owned groups (one wave each) -----------------------------------------
    const int own_n = TOPO ? s_ctl[28] : 0;
    const int own_base = TOPO ? s_ctl[29] : 0;
    const uint64_t topo_keys = own_n ? s_topo_keys : 0;
    const uint64_t b_keys = s_B.present | topo_keys;  // keys whose type filter must be redone on Add
    if (own_n) {
      for (int j = wave; j < own_n; j += NW) {
        const int oi = own_base + j;
        const int4 r0 = a.own_rec[2 * oi], r1 = a.own_rec[2 * oi + 1];  // the static part: one load
        const int g = r0.x, self = r0.y, k = r0.z, mskew = r0.w;
        uint64_t acc = 0;
        bool boot = false;  // pod affinity on a dictionary key: TopoOwn.self = bootstrap
        if (k >= 0) {
          const int c = a.tg_cnt[(size_t)g * 64 + lane];
          const uint64_t reg = a.tg_reg[g], pd = a.own_pd[oi];
          const bool sup = ((reg & pd) >> lane) & 1;
          const int mn = wave_min_i32(sup ? c : INT32_MAX);
          const int num = __builtin_popcountll(reg & pd);
          int64_t m = num ? (int64_t)mn : (int64_t)INT32_MAX;
          const int mind = r1.x;
          if (mind > 0 && num < mind) m = 0;
          if (mskew > 0) {  // spread: count + self - min <= maxSkew
            acc = __ballot(((reg >> lane) & 1) && (int64_t)c + self - m <= mskew);
          } else if (mskew == 0) {  // pod anti-affinity: known domains without a selected pod
            acc = __ballot(((reg >> lane) & 1) && c == 0);
          } else {  // pod affinity: known domains the pod admits that hold one; none: the self-selecting bootstrap
            acc = __ballot(sup && c > 0);
            boot = !acc && self;
            if (boot) acc = reg & pd;
          }
          s_tcnt[j][lane] = c;
          bytes += 64 * 4 + 16;
        }
        // pod affinity (hostname row, maxSkew -1): self = the pod may bootstrap (it selects itself and no domain
        // has a count yet, tg_reg bit 0)
        const int self_eff = mskew >= 0 ? self : k < 0 ? (self && !(a.tg_reg[g] & 1)) : (boot ? 1 : 0);
        if (lane == 0) {
          s_town[j] = TopoOwn{g, self_eff, k, r1.y, mskew, r1.z};
          s_tacc[j] = acc;
        }
      }
      __syncthreads();
    }

    // ---- addToExistingNode: lowest index whose CanAdd succeeds -------------------------------
    const int64_t ep0 = rmask_all ? s_preq[rr0] : 0, ep1 = rm1 ? s_preq[rr1] : 0;  // the pod, per headroom row
    const int64_t ep2 = rk2 >= 0 ? s_preq[rk2] : 0, ep3 = rk3 >= 0 ? s_preq[rk3] : 0;
    const uint64_t exd0 = EX_DIAG ? __builtin_amdgcn_s_memtime() : 0;
    if (EX_DIAG && tid == 0) g_sdiag[0] += exd0 - exdS;  // topology staging
    if (EX_DIAG && tid == 0 && s_ctl[17] < a.n_existing) g_sdiag[3] += 1;
    // the scan runs over list indices: every position, or (batched simulations) the shape-level's usable list
    const int32_t* ul = BATCH ? a.ex_ulist : nullptr;
    int u_base = 0, u_n = a.n_existing, u_start = s_ctl[17];
    if (ul) {
      u_base = a.ex_ulist_off[sl];
      u_n = a.ex_ulist_off[sl + 1] - u_base;
      u_start = u_start >= a.n_existing ? u_n : a.ex_uidx[(size_t)sl * a.n_existing + u_start];
    }
    for (int base = u_start; base < u_n && placed == -1 && !memo_fail; base += 4 * NT) {
      uint32_t flags = 0, iflags = 0;
      int pk[4];  // this thread's positions of the round (-1: past the list)
      const uint64_t exd1 = EX_DIAG ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {  // 4 rounds per thread: independent, so their loads overlap
        const int ix = base + k * NT + tid;
        pk[k] = ix < u_n ? (ul ? ul[u_base + ix] : ix) : -1;
        const int ec = pk[k];
        if (ec < 0) continue;
        // the failure memo: [shape-level][position], or (batched simulations) one entry per list entry
        const int32_t fl = a.ex_fail[ul ? (size_t)u_base + ix : (size_t)sl * a.n_existing + ec], ver = a.ex_ver[ec];
        const uint8_t sok = a.ex_static_ok[ec];
        const int32_t ts = a.ex_taintset[ec];
        // Fits(Merge(requests, pod), available), exact: unrequested resources never change. The headroom rows
        // (available - requests of the first four requested resources, [4][E]) coalesce across the positions.
        const size_t En = (size_t)a.n_existing;
        bool cand = a.ex_room[ec] >= ep0 && a.ex_room[En + ec] >= ep1;
        if (four) cand = cand && a.ex_room[2 * En + ec] >= ep2 && a.ex_room[3 * En + ec] >= ep3;
        cand = cand && fl != ver && fl != NC_NEVER && sok && ((tolmask >> ts) & 1);
        if (hpc) cand = cand && !(a.ex_hp[ec] & hpc);  // HostPortUsage.Conflicts (permanent: used bits only grow)
        if (rr_b4 && cand) {  // a fifth requested resource and beyond
          const int64_t* av = a.ex_available + (size_t)ec * KP_NRES;
          const int64_t* rq = a.ex_requests + (size_t)ec * KP_NRES;
          for (uint32_t rm = rr_b4; rm && cand; rm &= rm - 1) {
            const int r = __builtin_ctz(rm);
            cand = rq[r] + s_preq[r] <= av[r];
          }
        }
        // topology, exact: hostname: count + self <= maxSkew (min is 0 for hostname; the count only changes
        // when the node takes a pod, i.e. with its version); dictionary key: the node's domain is its label
        // value (or the key is undefined on it: incompatible), acceptable under the current counts
        for (int j = 0; j < own_n && cand; j++)
          if (s_town[j].key < 0) {
            const int c = (int)a.hcnt_ex[(size_t)s_town[j].row * a.n_existing + ec];
            cand = s_town[j].maxskew >= 0 ? c + s_town[j].self <= s_town[j].maxskew : (c > 0 || s_town[j].self);
          }
        if (cand) iflags |= 1u << k;  // passes everything that does not depend on the zone counts
        for (int j = 0; j < own_n && cand; j++) {
          const TopoOwn& o = s_town[j];
          if (o.key >= 0) {
            const uint8_t code = a.ex_tcode[(size_t)o.slot * a.n_existing + ec];
            cand = code != 0xFF && ((s_tacc[j] >> (code & 63)) & 1);
          }
        }
        flags |= (cand ? 1u : 0u) << k;
      }
      if (EX_DIAG) {  // the evaluation's cycles, as the slowest wave finishes them
        __syncthreads();
        if (tid == 0) g_sdiag[5] += __builtin_amdgcn_s_memtime() - exd1;
      }
      if (own_n) first_pos_min_e(iflags, pk, &s_ctl[24]);
      const int n = compact_candidates_x4e<NW>(flags, pk, s_list, s_wcnt, 0);
      if (wave == 0) bytes += (uint64_t)min(4 * NT, u_n - base) * (16 * a.n_req_res + 13);  // once
      const uint64_t exd2 = EX_DIAG ? __builtin_amdgcn_s_memtime() : 0;
      if (EX_DIAG && tid == 0) g_sdiag[1] += exd2 - exd1;
      for (int r0 = 0; r0 < n; r0 += NW) {
        const int li = r0 + wave;
        bool ok = false;
        uint64_t m_v = 0;
        ReqView rv;
        int ei = -1;
        if (li < n) {
          ei = s_list[li];
          attempts++;
          const KReqs* er = ex_req_src(a.ex_reqs, a.ex_reqs_ro, a.ex_own, ei);
          ok = merge_compatible(D, er, B, b_negop, false, m_v, rv, &slots[wave], vi);
          bytes += sizeof(KReqs);
          if (!ok && lane == 0)  // permanent unless the undefined-key rule failed (no well-known exemption here)
            a.ex_fail[ul ? (size_t)u_base + a.ex_uidx[(size_t)sl * a.n_existing + ei] : (size_t)sl * a.n_existing + ei] =
                (B->present & ~er->present & ~b_negop) == 0 ? NC_NEVER : a.ex_ver[ei];
          if (ok && own_n) ok = topo_narrow(D, own_n, s_town, s_tacc, s_tcnt, false, m_v, rv, vi);  // not memoised
        }
        if (lane == 0) s_ok[wave] = ok ? 1 : 0;
        __syncthreads();
        const int win = first_ok<NW>(s_ok);
        if (win >= 0) {
          if (wave == win) {
            store_merged(reinterpret_cast<KReqs*>(a.ex_reqs + (size_t)ei * sizeof(KReqs)), rv, m_v, D.W, D.KB);
            if (a.ex_reqs_ro && lane == 0) a.ex_own[ei >> 6] |= 1ull << (ei & 63);
            if (lane < KP_NRES) a.ex_requests[(size_t)ei * KP_NRES + lane] += s_preq[lane];
            if (lane < 4) {  // headroom rows of the first four requested resources
              const int64_t d = lane == 0 ? ep0 : lane == 1 ? ep1 : lane == 2 ? ep2 : ep3;
              a.ex_room[(size_t)lane * a.n_existing + ei] -= d;
            }
            if (lane == 0) a.ex_ver[ei] += 1;
            if (lane == 0 && hpa) a.ex_hp[ei] |= hpa;
          }
          placed = -2 - s_list[r0 + win];
        }
        __syncthreads();
        if (win >= 0) break;
      }
      if (EX_DIAG && tid == 0) g_sdiag[2] += __builtin_amdgcn_s_memtime() - exd2;
    }

    if (EX_DIAG && tid == 0) {
      g_sdiag[4] += __builtin_amdgcn_s_memtime() - exd0;
    }
    if (tid == 0 && a.n_existing) {
      // cursor: every position before the winner failed; with topology, before the first position that passed
      // the count-independent checks (a zone-count failure may pass later)
      const int cpos = own_n ? min(s_ctl[24], a.n_existing) : (placed != -1 ? -2 - placed : a.n_existing);
      a.cur_ex[2 * sl] = cpos;
      a.cur_ex[2 * sl + 1] = s_ctl[15];
      if (placed != -1) mstack_push((LdsI32)s_stk[1], (LdsI32)&s_ctl[14], (LdsI32)&s_ctl[21], ++s_ctl[15], -2 - placed);
    }
    TS(1);
    if (placed == -1) {
      int cmode = s_ctl[5];  // 1 LDS, 2 chunked, 0 flat global
      const ChkDir cd = chk_dir((int32_t LDS*)s_dyn);
      // ---- sort.Slice(newNodeClaims, len(Pods) asc) -----------------------------------------------
      // the cursor query (one lane of wave 1) overlaps the sort (thread 0); the pending mutation's own
      // clamp (s_ctl[16], known after the sort) is folded in below and pushed by thread 0 afterwards
      if (tid == 64) s_ctl[19] = min(s_ctl[22], mstack_query((LdsI32)s_stk[0], s_ctl[12], s_ctl[20], s_ctl[23]));
      if (cmode == 1) {
        sort_newnodeclaims<NT>((LdsI32)s_dyn, (LdsI32)(s_dyn + a.sort_cap), s_ctl[2], s_ctl[10], s_ctl[11], s_ctl, &a.stats[31]);
      } else if (cmode == 0) {
        sort_newnodeclaims<NT>((GlbI32)a.g_order, (GlbI32)a.g_npods, s_ctl[2], s_ctl[10], s_ctl[11], s_ctl, &a.stats[31]);
      } else {  // chunked: one wave replays the move on the blocks and the directory
        if (wave == 0) {
          const int low = chk_sort(cd, (ChkCtl LDS*)&g_chk, a.chk_blk, s_ctl[2], s_ctl[10], s_ctl[11], a.g_order, a.g_npods, &a.stats[31]);
          if (low == -3) chk_materialize(cd, (ChkCtl LDS*)&g_chk, a.chk_blk, a.g_order, a.g_npods);
          if (lane == 0) {
            s_ctl[18] = low;
            s_ctl[16] = low == -4 ? 0 : low;
            if (low <= -3) s_ctl[5] = 0;  // the directory is full: the flat order from here on
          }
        }
        __syncthreads();
        if (s_ctl[18] == -3)  // the pending mutation replays on the flat order
          sort_newnodeclaims<NT>((GlbI32)a.g_order, (GlbI32)a.g_npods, s_ctl[2], s_ctl[10], s_ctl[11], s_ctl, &a.stats[31]);
        cmode = s_ctl[5];
      }
      const bool in_lds = cmode == 1;
      const int n_nc = s_ctl[2];
      // a pod without requirements (at this level) merges into any NodeClaim without changing it: the append path
      // is exact on every candidate, tagged or not (NodeClaim.Add = Fits over the remaining types)
      const bool triv = s_B.present == 0;
      const int64_t p0 = rmask_all ? s_preq[rr0] : 0, p1 = rm1 ? s_preq[rr1] : 0;  // the pod, per record slot
      const int64_t p2 = rk2 >= 0 ? s_preq[rk2] : 0, p3 = rk3 >= 0 ? s_preq[rk3] : 0;
      const int start = res_strict ? 0 : min(min(s_ctl[19], s_ctl[16] >= 0 ? s_ctl[16] : INT32_MAX), n_nc);
      if (tid == 0) {
        s_ctl[10] = 0;
        if (s_ctl[16] >= 0) mstack_push((LdsI32)s_stk[0], (LdsI32)&s_ctl[12], (LdsI32)&s_ctl[20], ++s_ctl[13], s_ctl[16]);
      }
      TS(2);
      // ---- addToInflightNode: first NodeClaim in that order whose Add succeeds ------------------
      // chunked order: the scan walks the directory from the start position's chunk, skipping the chunks marked dead
      // for this shape-level (see chk_build); 4 x NW live chunks per iteration, one per wave and round
      __shared__ int32_t s_cw[2];
      if (cmode == 2) {
        if (wave == 0) {
          const int nch = g_chk.nch;
          const int c0 = start < n_nc ? chk_find(cd, nch, start) : nch;
          if (lane == 0) {
            s_cw[0] = c0;
            s_cw[1] = c0 < nch ? start - cd.start[c0] : 0;
          }
        }
        __syncthreads();
      }
      const int ch0 = cmode == 2 ? s_cw[0] : 0, cs0 = cmode == 2 ? s_cw[1] : 0;
      const bool can_dead = cmode == 2 && !own_n && !a.res_mode && sl < a.chk_dead_rows;
      int32_t* const deadrow = a.chk_dead + (size_t)(can_dead ? sl : 0) * CHK_MAXC;
      // entry in s_list of a candidate: its position (LDS / flat order) or chunk << 6 | slot (chunked order)
      auto ent_nc = [&](int e) -> int {
        e = LIST_POS(e);
        if (cmode == 1) return ((LdsI32)s_dyn)[e];
        if (cmode == 0) return ((GlbI32)a.g_order)[e];
        return a.chk_blk[ci_blk(cd.info[e >> 6])].id[e & 63];
      };
      auto ent_pos = [&](int e) -> int {
        e = LIST_POS(e);
        return cmode == 2 ? cd.start[e >> 6] + (e & 63) : e;
      };
      bool first_it = true;
      for (int base = start, cc = ch0; placed == -1 && !memo_fail;) {
        if (cmode == 2 ? cc >= g_chk.nch : base >= n_nc) break;
        uint32_t flags = 0, iflags = 0, tflags = 0, pf = 0;
        // 4 rounds per thread: independent, so their loads overlap. A spilled order (thousands of NodeClaims, long
        // scans bound by the gathers' cache-line traffic) first filters on the headroom of the first two requested
        // resources (one 16-byte load per position) and gathers the memo and the rest of the record for survivors.
        int ncs[4], pos[4], ent[4], tk[4];
        uint32_t room_ok = 0;
        int64_t r0s[4], r1s[4];
        int n_scan;
        if (cmode != 2) {
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int i = base + k * NT + tid;
            ncs[k] = i >= n_nc ? -1 : in_lds ? ((LdsI32)s_dyn)[i] : ((GlbI32)a.g_order)[i];
            pos[k] = ent[k] = i;
            tk[k] = -1;
          }
          n_scan = min(4 * NT, n_nc - base);
          base += 4 * NT;
        } else {
          // live chunks of the window [cc, cc + 64), in order (every wave computes the same mask); round k of wave w
          // takes the (k * NW + w)-th
          const int nch = g_chk.nch;
          const int b = ci_blk(cd.info[min(cc + lane, CHK_MAXC - 1)]);  // (unconditional, masked after)
          const bool dead = can_dead && deadrow[b] == cd.bep[b];
          const bool live = cc + lane < nch && !dead;
          uint64_t lm = __ballot(live);
          int nxt = min(cc + 64, nch);
          n_scan = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) tk[k] = -1;
          for (int j = 0; j < 4 * NW && lm; j++) {
            const int c = cc + __builtin_ctzll(lm);
            lm &= lm - 1;
            const int cnt = ci_cnt(cd.info[c]);
            n_scan += c == ch0 ? cnt - cs0 : cnt;
            if (j % NW == wave) tk[j / NW] = c;
            if (j == 4 * NW - 1 && lm) nxt = c + 1;
          }
          cc = nxt;
          if (n_scan == 0) continue;  // only dead chunks in this window
#pragma unroll
          for (int k = 0; k < 4; k++) {
            ncs[k] = -1;
            pos[k] = ent[k] = 0;
            const int c = tk[k];
            if (c < 0) continue;
            const uint32_t v = cd.info[c];
            if (lane < ci_cnt(v) && !(c == ch0 && lane < cs0)) {
              ncs[k] = a.chk_blk[ci_blk(v)].id[lane];
              pos[k] = cd.start[c] + lane;
              ent[k] = (c << 6) | lane;
            }
          }
        }
        if (cmode == 0) {
#pragma unroll
          for (int k = 0; k < 4; k++) {
            r0s[k] = r1s[k] = 0;
            if (ncs[k] < 0) continue;
            const int4 h = reinterpret_cast<const int4*>(a.nc_head + ncs[k])[0];
            r0s[k] = i64_of(h.x, h.y);
            r1s[k] = i64_of(h.z, h.w);
          }
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (ncs[k] >= 0 && r0s[k] >= p0 && r1s[k] >= p1) room_ok |= 1u << k;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (ncs[k] < 0 || (cmode == 0 && !((room_ok >> k) & 1))) continue;
          const int nc = ncs[k];
          // every gather is issued unconditionally so they overlap (one round trip instead of a chain)
          const int32_t fl = nc < a.ncc ? a.nc_fail[(size_t)sl * a.ncc + nc] : -2;
          const HeadView hv = load_head(a.nc_head + nc, four);
          const bool fit = hv.r0 >= p0 && hv.r1 >= p1 && hv.r2 >= p2 && hv.r3 >= p3;
          const bool tol = (tolmask >> hv.ts) & 1;
          const bool hpx = hpc && (a.nc_hp[nc] & hpc);
          // a permanent failure: headroom, taints and used host ports only get worse, NEVER stays (chunk dead marks)
          if (!fit || !tol || hpx || fl == NC_NEVER) pf |= 1u << k;
          bool cand = fit && tol && !hpx && fl != hv.ver && fl != NC_NEVER;
          if (rr_b4 && cand) {  // (a zero request holds trivially: requests <= max allocatable)
            const int64_t* rq = a.nc_requests + (size_t)nc * KP_NRES;
            const int64_t* mx = a.nc_maxalloc + (size_t)nc * KP_NRES;
            for (uint32_t rm = rr_b4; rm && cand; rm &= rm - 1) {
              const int r = __builtin_ctz(rm);
              if (s_preq[r] > 0) cand = rq[r] + s_preq[r] <= mx[r];
            }
          }
          for (int j = 0; j < own_n && cand; j++)  // hostname topologies, exact (count changes with the version)
            if (s_town[j].key < 0) {
              const int c = (int)a.hcnt_nc[(size_t)s_town[j].row * a.hnc_stride + nc];
              cand = s_town[j].maxskew >= 0 ? c + s_town[j].self <= s_town[j].maxskew : (c > 0 || s_town[j].self);
            }
          if (cand) iflags |= 1u << k;  // passes everything that does not depend on the zone counts
          bool pinned = true;  // every dictionary key the pod's groups spread over is one value on the NodeClaim
          for (int j = 0; j < own_n && cand; j++) {  // a NodeClaim pinned to one domain of a key can only take it
            const TopoOwn& o = s_town[j];
            if (o.key >= 0) {
              const uint8_t code = a.nc_tcode[(size_t)o.slot * a.hnc_stride + nc];
              cand = code == 0xFF || (code < 64 && ((s_tacc[j] >> (code & 63)) & 1));
              pinned = pinned && code < 64;
            }
          }
          // shape-level already merged: the append path (Fits alone). With topology groups only when the NodeClaim is
          // pinned on their keys: topo_narrow then keeps its requirements (the acceptable domain is its own value,
          // tested above; hostname rows exactly by the counts), so the Add changes nothing but requests and types
          if (cand && (fl >= NC_MERGED || triv) && !a.res_mode && (!own_n || pinned)) tflags |= 1u << k;
          flags |= (cand ? 1u : 0u) << k;
        }
        if (own_n) first_pos_min_e(iflags, pos, &s_ctl[25]);
        if (can_dead) {  // a chunk scanned in full whose NodeClaims all failed permanently: dead for this shape-level
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int c = tk[k];
            if (c < 0 || (c == ch0 && cs0 > 0)) continue;
            if (__ballot(ncs[k] >= 0 && !((pf >> k) & 1)) == 0 && lane == 0) {
              const int b = ci_blk(cd.info[c]);
              deadrow[b] = cd.bep[b];
            }
          }
        }
        if (tid == 0) {
          scanned += n_scan;
          if (first_it) starts += start;
        }
        first_it = false;
        const int n = compact_candidates_x4e<NW>(flags, ent, s_list, s_wcnt, tflags);
        TS(6);
        if (wave == 0) bytes += (uint64_t)n_scan * (12 + 16 * a.n_req_res);  // counted once
        // a round whose first candidate takes the append path evaluates it alone (it is the likely winner and
        // costs a fraction of a full attempt, which the other waves would make the round wait for)
        for (int r0 = 0, width = NW; r0 < n; r0 += width) {
          width = (s_list[r0] & LIST_TAG) ? 1 : NW;
          const int li = r0 + wave;
          bool ok = false, fast = false, perm = true;
          uint64_t m_v = 0, X = 0, held = 0, nh = 0;
          ReqView rv;
          int nc = -1;
          if (wave < width && li < n) {
            nc = ent_nc(s_list[li]);
            attempts++;
            uint64_t* tsub = (a.timing && wave == 0) ? s_tsub : nullptr;
            const uint64_t tm0 = tsub ? __builtin_amdgcn_s_memtime() : 0;
            // one batch of independent loads: the candidate's requirements, remaining types, requests, cached
            // threshold indices and catalogue; everything after it is LDS/ALU until filter_types' row batch
            const CandReq cr = load_cand(D, kreq_at(a.nc_reqs, nc));
            const int cat = a.nc_cat[nc];
            const uint64_t X0 = lane < D.TW ? a.nc_X[(size_t)nc * D.TW + lane] : 0;
            const int64_t rq_lane = lane < KP_NRES ? a.nc_requests[(size_t)nc * KP_NRES + lane] : 0;
            const int32_t j0_lane = lane < KP_NRES ? a.nc_fitj[(size_t)nc * KP_NRES + lane] : 0;
            fast = (s_list[li] & LIST_TAG) && !(cr.hmin & cr.P);
            if (fast) {
              const int64_t q_lane = rq_lane + (lane < KP_NRES ? s_preq[lane] : 0);
              X = fits_filter(D, hdr(cat), X0, q_lane, j0_lane, (const int64_t LDS*)s_fitv, a.req_res_mask,
                              (RowPtr LDS*)s_rl[wave], &bytes, s_fitj[wave]);
              ok = __ballot(X != 0) != 0;
              bytes += (uint64_t)D.TW * 8 + KP_NRES * 8 + 8;
            } else {
              ok = merge_compatible(D, cr, B, b_negop, true, m_v, rv, &slots[wave], vi);
              if (!ok) perm = (B->present & ~cr.P & ~b_negop & ~D.wellknown) == 0;
              bytes += sizeof(KReqs);
            }
            if (tsub && lane == 0) tsub[0] += __builtin_amdgcn_s_memtime() - tm0;
            bool memo = !ok || !own_n;  // failures after the topology step depend on the counts
            if (ok && own_n && !fast) ok = topo_narrow(D, own_n, s_town, s_tacc, s_tcnt, true, m_v, rv, vi);
            if (ok && !fast) {
              const int pb = cat < 32 ? s_pvpb[cat] : a.pvp_base[sl * a.n_catalogs + cat];
              const uint64_t* pvp = a.shape_pvp + (size_t)pb * D.TW;
              const int64_t q_lane = rq_lane + (lane < KP_NRES ? s_preq[lane] : 0);
              X = filter_types(D, hdr(cat), rv, m_v, X0, b_keys, pvp, s_pslot, q_lane, j0_lane, (const int64_t LDS*)s_fitv,
                               a.req_res_mask, vi, s_scratch[wave], (RowPtr LDS*)s_rl[wave], &bytes, s_fitj[wave], topo_keys, tsub);
              ok = __ballot(X != 0) != 0;
              if (tsub && lane == 0) tsub[5] += 1;  // attempts reaching filter_types (wave 0)
              bytes += (uint64_t)D.TW * 8 + KP_NRES * 8;
            }
            if (ok && a.res_mode) {  // reserveOfferings: a strict failure depends on the capacities (not memoised)
              held = a.nc_held[nc];
              nh = reserve_classes(D, hdr(cat), rv, m_v, X, a.res_cls, held, (const int32_t LDS*)s_rcap, res_strict, vi);
              if (nh == ~0ull) ok = memo = false;
            }
            if (!ok && memo && lane == 0 && nc < a.ncc) a.nc_fail[(size_t)sl * a.ncc + nc] = perm ? NC_NEVER : a.nc_head[nc].ver;
          }
          if (lane == 0 && wave < width) s_ok[wave] = ok ? 1 : 0;
          __syncthreads();
          TS(7);
          const int win = width == 1 ? (s_ok[0] ? 0 : -1) : first_ok<NW>(s_ok);
          if (win >= 0) {
            if (wave == win) {
              if (!fast) {  // the append path leaves the requirements as they are
                store_merged(reinterpret_cast<KReqs*>(a.nc_reqs + (size_t)nc * sizeof(KReqs)), rv, m_v, D.W, D.KB);
                if (a.n_tk) store_tcodes(a.n_tk, a.tk_keys, a.nc_tcode, a.hnc_stride, rv, m_v, nc);
              }
              if (lane == 0 && nc < a.ncc) a.nc_fail[(size_t)sl * a.ncc + nc] = NC_MERGED;  // (count-independent)
              if (lane < D.TW) a.nc_X[(size_t)nc * D.TW + lane] = X;
              if (lane < KP_NRES) a.nc_requests[(size_t)nc * KP_NRES + lane] += s_preq[lane];
              if (lane == 0 && hpa) a.nc_hp[nc] |= hpa;
              if (lane == 0) {
                if (in_lds) {
                  ((LdsI32)(s_dyn + a.sort_cap))[nc] += 1;
                } else {
                  ((GlbI32)a.g_npods)[nc] += 1;
                  if (cmode == 2) {  // len(Pods) in the NodeClaim's block as well (the sort replay reads it there)
                    const int e = LIST_POS(s_list[li]);
                    a.chk_blk[ci_blk(cd.info[e >> 6])].key[e & 63] += 1;
                  }
                }
                NcHead* h = a.nc_head + nc;
                h->ver += 1;
                h->room[0] -= p0;
                h->room[1] -= p1;
                h->room[2] -= p2;
                h->room[3] -= p3;
              }
              if (lane < KP_NRES) a.nc_fitj[(size_t)nc * KP_NRES + lane] = s_fitj[wave][lane];
              if (a.res_mode) {
                reserve_commit((int32_t LDS*)s_rcap, held, nh);
                if (lane == 0) a.nc_held[nc] = nh;
              }
            }
            const int wpos = ent_pos(s_list[r0 + win]);
            placed = ent_nc(s_list[r0 + win]);
            if (tid == 0) {
              s_ctl[10] = 1;
              s_ctl[11] = wpos;
              // cursor: all positions before the winner failed (topology: before the first count-independent pass)
              a.cur_nc[2 * sl] = own_n ? min(s_ctl[25], wpos) : wpos;
              a.cur_nc[2 * sl + 1] = s_ctl[13];
            }
          }
          __syncthreads();
          if (win >= 0) break;
        }
      }
    }

    TS(3);
    if (placed == -1) {
      if (tid == 0) {  // every in-flight NodeClaim failed
        a.cur_nc[2 * sl] = own_n ? min(s_ctl[25], s_ctl[2]) : s_ctl[2];
        a.cur_nc[2 * sl + 1] = s_ctl[13];
      }
      // ---- addToNewNodeClaim: templates in weight order --------------------------------------------
      for (int base = 0; base < a.n_tmpl && placed == -1 && !memo_fail; base += NT) {
        const int t = base + tid;
        // a memoised failure is permanent: remaining limits only shrink, and the rest is a function of the
        // (template, shape-level) pair (failures that depend on topology counts or reservations are not memoised)
        const bool cand = t < a.n_tmpl && ((tolmask >> a.tmpl_taintset[t]) & 1) &&
                          a.tmpl_fail[(size_t)sl * a.n_tmpl + t] != NC_NEVER;
        const int n = compact_candidates<NW>(cand, t, s_list, s_wcnt);
        for (int r0 = 0; r0 < n; r0 += NW) {
          if (FX_DIAG && tid == 0) g_sdiag[4] += 1;  // diagnostic: template rounds
          const int li = r0 + wave;
          bool ok = false;
          uint64_t m_v = 0, X = 0, nh = 0;
          ReqView rv;
          int tm = -1;
          if (li < n) {
            tm = s_list[li];
            const int cat = a.tmpl_catalog[tm];
            const CatHdr LDS* H = hdr(cat);
            X = lane < D.TW ? a.tmpl_X[(size_t)tm * D.TW + lane] : 0;
            const uint32_t lim = a.tmpl_limit_present[tm];
            if (lim) {  // filterByRemainingResources: capacity <= remaining for every limited resource
              const int32_t ver = a.tmpl_ver[tm];
              if (a.tmpl_xlim_ver[tm] == ver) {  // computed since the last subtractMax on this template
                X = lane < D.TW ? a.tmpl_xlim[(size_t)tm * D.TW + lane] : 0;
              } else {
                // lane l tests type 64 i + l of word i (coalesced capacity rows, independent loads across words)
                const int64_t* rem = a.tmpl_remaining + (size_t)tm * KP_NRES;
                uint64_t keep = 0;
                for (int i = 0; i < D.TW; i++) {
                  const uint64_t w = lane_bcast(X, i);
                  if (!w) continue;
                  const int ty = i * 64 + lane;
                  bool viable = ((w >> lane) & 1) && ty < D.T;
                  for (uint32_t rm = lim; rm && viable; rm &= rm - 1) {
                    const int r = __builtin_ctz(rm);
                    viable = H->d.cap[(size_t)r * D.T + ty] <= rem[r];
                  }
                  const uint64_t bal = __ballot(viable);
                  if (lane == i) keep = bal;
                }
                X = keep;
                if (lane < D.TW) a.tmpl_xlim[(size_t)tm * D.TW + lane] = X;
                if (lane == 0) a.tmpl_xlim_ver[tm] = ver;
              }
              bytes += (uint64_t)D.T * 8;
            }
            bool memo = true;
            if (__ballot(X != 0)) {
              attempts++;
              const int64_t q_lane = lane < KP_NRES ? a.tmpl_daemon[(size_t)tm * KP_NRES + lane] + s_preq[lane] : 0;
              ok = merge_compatible(D, kreq_at(a.tmpl_reqs, tm), B, b_negop, true, m_v, rv, &slots[wave], vi);
              memo = !ok || !own_n;
              if (ok && own_n) ok = topo_narrow(D, own_n, s_town, s_tacc, s_tcnt, true, m_v, rv, vi);
              for (int j = 0; j < own_n && ok; j++)  // a fresh node has no count: pod affinity only by bootstrap
                if (s_town[j].key < 0 && s_town[j].maxskew < 0 && !s_town[j].self) ok = false;
              if (ok && a.tfeas && !own_n) {
                // the template's types for this shape-level, precomputed (tmpl_feas_kernel, row-sharded over ranks):
                // filter_types is a per-type filter, so (options after the limits) ∩ (filtered template) is the
                // filtered set; minValues is a property of the set and is checked on the intersection
                const uint64_t* e = a.tfeas + ((size_t)sl * a.n_tmpl + tm) * a.tfeas_words;
                X &= lane < D.TW ? e[lane] : 0;
                if (lane < KP_NRES) s_fitj[wave][lane] = reinterpret_cast<const int32_t*>(e + D.TW)[lane];
                if (rv.hmin & rv.present)
                  if (!minvalues_ok(D, H->d.code, H->d.TM, rv.hmin & rv.present, rv.minv, X, s_scratch[wave])) X = 0;
                bytes += (uint64_t)D.TW * 8 + KP_NRES * 4;
                ok = __ballot(X != 0) != 0;
              } else if (ok) {
                const int pb = cat < 32 ? s_pvpb[cat] : a.pvp_base[sl * a.n_catalogs + cat];
                const uint64_t* pvp = a.shape_pvp + (size_t)pb * D.TW;
                X = filter_types(D, H, rv, m_v, X, b_keys, pvp, s_pslot, q_lane, 0, (const int64_t LDS*)s_fitv, a.req_res_mask, vi,
                                 s_scratch[wave], (RowPtr LDS*)s_rl[wave], &bytes, s_fitj[wave], topo_keys);
                ok = __ballot(X != 0) != 0;
              }
              if (ok && a.res_mode) {  // a new NodeClaim holds nothing yet
                nh = reserve_classes(D, H, rv, m_v, X, a.res_cls, 0, (const int32_t LDS*)s_rcap, res_strict, vi);
                if (nh == ~0ull) {
                  ok = memo = false;
                  if (lane == 0) s_ctl[27] = 1;  // ReservedOfferingError: the pod is not relaxed
                }
              }
            }
            if (!ok && memo && lane == 0) a.tmpl_fail[(size_t)sl * a.n_tmpl + tm] = NC_NEVER;
          }
          if (lane == 0) s_ok[wave] = ok ? 1 : 0;
          __syncthreads();
          const int win = first_ok<NW>(s_ok);
          const int nc = s_ctl[2];
          const int cmode = s_ctl[5];
          const bool in_lds = cmode == 1;
          if (win >= 0) {
            if (wave == win) {
              store_merged(reinterpret_cast<KReqs*>(a.nc_reqs + (size_t)nc * sizeof(KReqs)), rv, m_v, D.W, D.KB);
              if (a.n_tk) store_tcodes(a.n_tk, a.tk_keys, a.nc_tcode, a.hnc_stride, rv, m_v, nc);
              if (lane < D.TW) a.nc_X[(size_t)nc * D.TW + lane] = X;
              if (lane < KP_NRES)
                a.nc_requests[(size_t)nc * KP_NRES + lane] = a.tmpl_daemon[(size_t)tm * KP_NRES + lane] + s_preq[lane];
              if (lane == 0) {
                a.nc_tmpl[nc] = tm;
                a.nc_cat[nc] = a.tmpl_catalog[tm];
                if (a.hp_any) a.nc_hp[nc] = hpa;  // a template's HostPortUsage is empty
              }
              if (lane < KP_NRES) a.nc_fitj[(size_t)nc * KP_NRES + lane] = s_fitj[wave][lane];
              if (lane == 0 && nc < a.ncc) a.nc_fail[(size_t)sl * a.ncc + nc] = NC_MERGED;
              if (a.res_mode) {
                reserve_commit((int32_t LDS*)s_rcap, 0, nh);
                if (lane == 0) a.nc_held[nc] = nh;
              }
              const uint64_t fxd0 = FX_DIAG ? __builtin_amdgcn_s_memtime() : 0;
              store_maxalloc(hdr(a.tmpl_catalog[tm])->d.alloc, lane < D.TW ? X : 0, D.T, a.req_res_mask,
                             a.nc_maxalloc + (size_t)nc * KP_NRES, a.nc_head + nc,
                             lane < KP_NRES ? a.tmpl_daemon[(size_t)tm * KP_NRES + lane] + s_preq[lane] : 0,
                             a.tmpl_taintset[tm]);
              // subtractMax: remaining -= max capacity over the new NodeClaim's InstanceTypeOptions
              const uint32_t lim = a.tmpl_limit_present[tm];
              if (lim) {
                const CatHdr LDS* Hc = hdr(a.tmpl_catalog[tm]);
                for (int r = 0; r < KP_NRES; r++) {
                  if (!((lim >> r) & 1)) continue;
                  const int64_t mx = max_over_types(Hc->d.cap + (size_t)r * D.T, lane < D.TW ? X : 0, D.TW, D.T);
                  if (lane == 0) a.tmpl_remaining[(size_t)tm * KP_NRES + r] -= mx;
                }
                if (lane == 0) a.tmpl_ver[tm] += 1;
              }
              if (FX_DIAG && lane == 0) g_sdiag[5] += __builtin_amdgcn_s_memtime() - fxd0;  // diagnostic
            }
            placed = nc;
          }
          __syncthreads();
          if (win >= 0) {
            // append to newNodeClaims: past a.sort_cap the sort arrays leave LDS for the chunked order (or, when its
            // directory cannot hold them, the flat global arrays)
            const bool spill = in_lds && nc == a.sort_cap;
            if (spill) {
              for (int i = tid; i < nc; i += NT) {
                a.g_order[i] = s_dyn[i];
                a.g_npods[i] = s_dyn[a.sort_cap + i];
              }
            }
            __syncthreads();
            const ChkDir cd = chk_dir((int32_t LDS*)s_dyn);
            if (spill && wave == 0) {
              const bool ok = chk_build(cd, (ChkCtl LDS*)&g_chk, a.chk_blk, a.g_order, a.g_npods, nc);
              if (lane == 0) s_ctl[5] = ok ? 2 : 0;
            }
            __syncthreads();
            if (s_ctl[5] == 2) {
              if (wave == 0) {
                if (lane == 0) a.g_npods[nc] = 1;
                if (!chk_append(cd, (ChkCtl LDS*)&g_chk, a.chk_blk, nc, 1)) {  // the directory is full: the flat order
                  chk_materialize(cd, (ChkCtl LDS*)&g_chk, a.chk_blk, a.g_order, a.g_npods);
                  if (lane == 0) {
                    a.g_order[nc] = nc;
                    s_ctl[5] = 0;
                  }
                }
                if (lane == 0) {
                  s_ctl[2] = nc + 1;
                  s_ctl[10] = 2;
                }
              }
            } else if (tid == 0) {
              const bool lds_now = s_ctl[5] == 1;
              int32_t* ord = lds_now ? s_dyn : a.g_order;
              int32_t* npods = lds_now ? s_dyn + a.sort_cap : a.g_npods;
              ord[nc] = nc;
              npods[nc] = 1;
              s_ctl[2] = nc + 1;
              s_ctl[10] = 2;
            }
            break;
          }
        }
      }
    }

    // ---- Topology.Record: every group selecting the pod whose node filter admits the node counts it
    //      in the node's domain (dictionary keys: only once the key is a single value) -------------
    if (TOPO && placed != -1 && wave == 0) {
      // lane i takes the i-th group: the groups' attributes are gathered together, and each lane updates its own
      // group's counts (distinct groups: no two lanes touch one counter); node-filter terms go through the wave
      const int rn = a.shape_rec_n[shape];
      const int rb = a.shape_rec_base[shape];
      const bool ex = placed <= -2;
      const int idx = ex ? -2 - placed : placed;
      const KReqs* fin = ex ? ex_req_src(a.ex_reqs, a.ex_reqs_ro, a.ex_own, idx) : kreq_at(a.nc_reqs, idx);
      const int ts = ex ? a.ex_taintset[idx] : a.nc_head[idx].taintset;
      for (int i0 = 0; i0 < rn; i0 += 64) {
        const int i = i0 + lane;
        const bool act = i < rn;
        const int g = act ? a.rec_list[rb + i] : 0;
        bool ok = act && a.tg_live[g] && ((a.tg_filt_tol[g] >> ts) & 1);
        const int row = act ? a.tg_row[g] : -1;
        const int k = act ? a.tg_key[g] : 0;
        const int mskew = act ? a.tg_maxskew[g] : 0;
        uint64_t need = __ballot(ok && a.tg_aff[g]);
        while (need) {  // TopologyNodeFilter.MatchesRequirements: Compatible(node reqs, some term)
          const int l = __builtin_ctzll(need);
          need &= need - 1;
          const int gg = __builtin_amdgcn_readlane(g, l);
          const int tb = a.tg_term_base[gg], nt = a.tg_nterm[gg];
          bool m = false;
          for (int ti = 0; ti < nt && !m; ti++) {
            uint64_t mv;
            ReqView rv;
            m = merge_compatible(D, fin, kreq_at(a.tg_terms, tb + ti), a.tg_terms_negop[tb + ti], !ex, mv, rv, &slots[0], vi);
          }
          if (lane == l) ok = m;
        }
        if (ok) {
          if (row >= 0) {
            uint8_t* c = ex ? &a.hcnt_ex[(size_t)row * a.n_existing + idx] : &a.hcnt_nc[(size_t)row * a.hnc_stride + idx];
            *c = *c == 255 ? 1 : *c < 254 ? *c + 1 : 254;  // 255: an unregistered domain (Record registers it)
            a.tg_reg[g] = 1;  // hostname rows: some domain has a count (ends pod-affinity bootstrap)
          } else {
            const uint64_t v = fin->vals[k];
            const bool has = (fin->present >> k) & 1;
            if (mskew == 0) {  // pod anti-affinity: Record(domains.Values()...), every value of the key
              if (has) {
                for (uint64_t m = v; m; m &= m - 1) a.tg_cnt[(size_t)g * 64 + __builtin_ctzll(m)] += 1;
                a.tg_reg[g] |= v;
              }
            } else if (has && !((fin->compl_ >> k) & 1) && __builtin_popcountll(v) == 1) {
              const int d = __builtin_ctzll(v);
              a.tg_cnt[(size_t)g * 64 + d] += 1;
              a.tg_reg[g] |= 1ull << d;
            }
          }
        }
        bytes += 16 * (uint64_t)min(64, rn - i0);
      }
    }  // (the bookkeeping barrier below publishes the counts before the next pod stages them)
    TS(4);
    // ---- bookkeeping (thread 0): placement, or Preferences.Relax + Queue.Push -------------------
    if (tid == 0) {
      if (placed != -1) {
        a.placement[pod] = placed;
        a.events[s_ctl[4]++] = pod;
      } else {
        a.placement[pod] = -1;
        if (!TOPO && !a.res_mode && (s_B.present & ~b_negop & ~D.wellknown) == 0) a.sl_fail[sl] = s_ctl[2];
        const bool res_err = s_ctl[27] != 0;  // a ReservedOfferingError is not relaxed (upstream trySchedule)
        if (res_err) a.stats[40] += 1;
        const bool relaxed = !res_err && lvl + 1 < a.shape_nlevels[shape];
        if (relaxed) a.pod_level[pod] = lvl + 1;
        if (TOPO && relaxed) {  // Topology.Update: the groups the relaxed pod owns now exist from here on
          const int nsl = sl + 1;
          for (int i = 0; i < a.sl_own_n[nsl]; i++) {
            const int g = a.own_group[a.sl_own_base[nsl] + i];
            if (a.tg_live[g]) continue;
            a.tg_live[g] = 1;
            // a new hostname group: the NodeClaims created before it were never registered with it (Register runs
            // at NodeClaim creation over the groups that exist then)
            const int row = a.tg_row[g];
            if (row >= 0)
              for (int x = 0; x < s_ctl[2]; x++) a.hcnt_nc[(size_t)row * a.hnc_stride + x] = 255;
          }
        }
        int len = s_ctl[1];
        int tail = s_ctl[0] + len;
        if (tail >= a.n_pods) tail -= a.n_pods;
        a.queue[tail] = pod;
        len += 1;
        s_ctl[1] = len;
        if (relaxed) {
          s_ctl[3] += 1;  // lastLen = map{}
        } else {
          a.lastlen[pod] = len;
          a.lastlen_epoch[pod] = s_ctl[3];
        }
      }
    }
    __syncthreads();
    TS(5);
  }
#undef TS
  if (timing)
    for (int i = 0; i < 8; i++) a.stats[8 + i] = tph[i], a.stats[16 + i] = s_tsub[i];

  if (lane == 0) {
    atomicAdd((unsigned long long*)&a.stats[0], (unsigned long long)attempts);
    atomicAdd((unsigned long long*)&a.stats[1], (unsigned long long)bytes);
  }
  if (tid == 0) {
    a.stats[2] = pops;
    a.stats[3] = (uint64_t)s_ctl[2];
    a.stats[4] = (uint64_t)s_ctl[4];
    a.stats[5] = scanned + g_fast.scanned;  // in-flight positions scanned by the pre-pass
    a.stats[6] = starts + g_fast.starts;    // sum of cursor start positions
    atomicAdd((unsigned long long*)&a.stats[0], (unsigned long long)g_fast.attempts);
    atomicAdd((unsigned long long*)&a.stats[1], (unsigned long long)g_fast.bytes);
    a.stats[24] = g_fast.fpods;
    for (int i = 0; i < 8; i++) a.stats[32 + i] = g_fast.fbail[i];
    for (int i = 0; i < 6; i++) a.stats[25 + i] = g_fast.fcyc[i];
    if (FT_FINE && timing)
      for (int i = 0; i < 8; i++) a.stats[16 + i] = g_fast.fcyc[6 + i];
    if (SORT_DIAG || EX_DIAG || FX_DIAG)
      for (int i = 0; i < 6; i++) a.stats[25 + i] = g_sdiag[i];
    // chunked order: peak chunks, splits, emptied chunks, (re)builds; final order mode
    a.stats[41] = g_chk.nch_peak;
    a.stats[42] = g_chk.splits;
    a.stats[43] = g_chk.removals;
    a.stats[44] = g_chk.rebuilds;
    a.stats[45] = s_ctl[5];
    a.stats[47] = g_fast.runpods;
  }
  if (s_ctl[5] == 1)
    for (int i = tid; i < s_ctl[2]; i += NT) {
      a.g_npods[i] = s_dyn[a.sort_cap + i];
      a.g_order[i] = s_dyn[i];
    }
}

// ------------------------------------------------------------------------------------------------
// tmpl_feas_kernel: for each (shape-level, NodePool template) pair of a row range, the template's InstanceTypeOptions
// a new NodeClaim for that shape-level would start from (addToNewNodeClaim: Compatible + Add of the requirements,
// then filterInstanceTypesByRequirements over the template's types with the daemon + pod requests), without the
// NodePool limits and minValues, which solve_kernel applies at use. Entry (tfeas_words u64): the type mask, the Fits
// threshold indices (int32 x KP_NRES), and a word: 1 compatible / 0 incompatible / -1 not precomputed (shape-levels
// that own topology groups narrow the requirements by the current counts first). One wave per pair. Row ranges are
// what the ranks of a kp_comm split between them before one ncclAllGather of the table.
// ------------------------------------------------------------------------------------------------
#define TF_WAVES 4
__global__ __launch_bounds__(TF_WAVES * 64) void tmpl_feas_kernel(TfeasArgs a) {
  __shared__ DevDict D;
  __shared__ WaveSlots slots[TF_WAVES];
  __shared__ uint32_t s_scratch[TF_WAVES][2 * KP_MAX_WORDS];
  __shared__ RowPtr s_rl[TF_WAVES][RL_CAP];
  __shared__ int32_t s_fitj[TF_WAVES][KP_NRES];
  __shared__ CatHdr s_hdr[TF_WAVES];
  __shared__ int64_t s_vint[KP_MAX_BOUND_KEYS * 64];
  block_copy(D, a.dict);
  __syncthreads();
  for (int i = threadIdx.x; i < D.KB * 64; i += TF_WAVES * 64) s_vint[i] = a.vint[i];
  __syncthreads();
  const VInt vi{(const int64_t LDS*)s_vint, a.vint, D.KB};
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = LANE;
  const int NTm = a.n_tmpl, TW = D.TW;
  const long first = (long)a.row_lo * NTm, last = (long)a.row_hi * NTm;
  for (long pr = first + (long)blockIdx.x * TF_WAVES + wave; pr < last; pr += (long)gridDim.x * TF_WAVES) {
    const int sl = (int)(pr / NTm), t = (int)(pr % NTm);
    uint64_t* e = a.out + (size_t)pr * a.words;
    int32_t* ej = reinterpret_cast<int32_t*>(e + TW);
    if (a.sl_own_n[sl] > 0) {
      if (lane == 0) e[TW + KP_NRES / 2] = (uint64_t)(int64_t)-1;
      continue;
    }
    const int shape = a.sl_shape[sl];
    const int cat = a.tmpl_catalog[t];
    hdr_fill_wave((CatHdr LDS*)&s_hdr[wave], &a.cats[cat], D.C);
    wave_sync();
    const CatHdr LDS* H = (const CatHdr LDS*)&s_hdr[wave];
    const KReqs* B = kreq_at(a.shape_reqs, sl);
    uint64_t m_v = 0;
    ReqView rv;
    const bool ok = merge_compatible(D, kreq_at(a.tmpl_reqs, t), B, a.shape_negop[sl], true, m_v, rv, &slots[wave], vi);
    uint64_t X = 0;
    int32_t j_lane = 0;
    if (ok) {
      X = lane < TW ? a.tmpl_X[(size_t)t * TW + lane] : 0;
      const uint64_t* pvp = a.shape_pvp + (size_t)a.pvp_base[sl * a.n_catalogs + cat] * TW;
      const int64_t q_lane = lane < KP_NRES ? a.tmpl_daemon[(size_t)t * KP_NRES + lane] +
                                                  a.shape_requests[(size_t)shape * KP_NRES + lane]
                                            : 0;
      uint64_t bytes = 0;
      X = filter_types(D, H, rv, m_v, X, B->present, pvp, a.pvp_slot + (size_t)sl * KP_MAX_KEYS, q_lane, 0, nullptr,
                       a.req_res_mask, vi, s_scratch[wave], (RowPtr LDS*)s_rl[wave], &bytes, s_fitj[wave], 0, nullptr,
                       false);
      j_lane = lane < KP_NRES ? s_fitj[wave][lane] : 0;
    }
    if (lane < TW) e[lane] = X;
    if (lane < KP_NRES) ej[lane] = j_lane;
    if (lane == 0) e[TW + KP_NRES / 2] = ok ? 1 : 0;
  }
}

hipError_t launch_tmpl_feas(const TfeasArgs& a, hipStream_t s) {
  const long pairs = (long)(a.row_hi - a.row_lo) * a.n_tmpl;
  if (pairs <= 0) return hipSuccess;
  const int blocks = (int)std::min<long>((pairs + TF_WAVES - 1) / TF_WAVES, 4096);
  hipLaunchKernelGGL(tmpl_feas_kernel, dim3(blocks), dim3(TF_WAVES * 64), 0, s, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// finalize_kernel: one workgroup per NodeClaim. OrderByPrice(reqs) + Truncate(max).
// ------------------------------------------------------------------------------------------------
#define FIN_THREADS 256
#define FIN_MAX_T 4096
// BATCH: workgroup y finalizes NodeClaim 0 of simulation y (batch[y]) when that Solve made exactly one NodeClaim (the
// only case a consolidation decision reads options from), its count read from the Solve's stats on the device.
template <bool BATCH>
__global__ __launch_bounds__(FIN_THREADS) void finalize_kernel(FinalizeArgs a0, const FinalizeArgs* __restrict__ batch) {
  __shared__ DevDict D;
  __shared__ uint64_t s_cls;
  __shared__ uint64_t s_key[FIN_MAX_T];
  __shared__ uint32_t s_idx[FIN_MAX_T];
  __shared__ uint32_t s_cnt;
  const FinalizeArgs& a = BATCH ? batch[blockIdx.x] : a0;
  if (BATCH && a.solve_stats[3] != 1) return;
  const int nc = BATCH ? 0 : blockIdx.x;
  block_copy(D, a.dict);
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const int tm = a.nc_tmpl[nc];
  const DevCatalog& Cg = a.cats[a.tmpl_catalog[tm]];
  const KReqs* R = reinterpret_cast<const KReqs*>(a.nc_reqs + (size_t)nc * sizeof(KReqs));
  if (threadIdx.x < 64) {  // wave 0: offering classes compatible with the final requirements
    const int lane = LANE;
    const uint64_t v = lane < D.W ? R->vals[lane] : 0;
    ReqView rv;
    rv.present = R->present;
    rv.compl_ = R->compl_ & R->present;
    rv.hgt = R->hgt;
    rv.hlt = R->hlt;
    rv.hmin = R->hmin;
    rv.nz = nz_keys(D, v);
    rv.dne = 0;
    rv.gt = R->gt;
    rv.lt = R->lt;
    rv.minv = R->minv;
    const uint64_t negR = negop_mask(rv.present, rv.compl_, rv.nz);
    const uint64_t allowed = allowed_word(D, rv, v, vint_global(a.vint));
    uint64_t cls = allowed_classes(D, Cg.cls, rv, allowed, negR);
    const uint64_t held = a.nc_held ? a.nc_held[nc] : 0;
    if (held) cls &= held;  // FinalizeScheduling: reservation-id In {held ids}
    if (lane == 0) s_cls = cls;
  }
  __syncthreads();
  const uint64_t cls = s_cls;
  for (int t = threadIdx.x; t < D.T; t += FIN_THREADS) {
    const uint64_t xw = a.nc_X[(size_t)nc * D.TW + (t >> 6)];
    if (!((xw >> (t & 63)) & 1)) continue;
    double p = __builtin_huge_val();
    uint64_t m = cls;
    if (Cg.price_sub) {  // min over the compatible class set in one gather
      p = Cg.price_sub[(size_t)cls * D.T + t];
      m = 0;
    }
    while (m) {
      const int c = __builtin_ctzll(m);
      m &= m - 1;
      const double q = Cg.price_cm[(size_t)c * D.T + t];
      p = q < p ? q : p;
    }
    const uint32_t slot = atomicAdd(&s_cnt, 1u);
    s_key[slot] = (uint64_t)__double_as_longlong(p);  // non-negative doubles order like their bits
    s_idx[slot] = (Cg.name_rank[t] << 12) | (uint32_t)t;
  }
  __syncthreads();
  const uint32_t n = s_cnt;
  uint32_t n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (uint32_t i = n + threadIdx.x; i < n2; i += FIN_THREADS) {
    s_key[i] = ~0ull;
    s_idx[i] = ~0u;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= n2; k <<= 1) {  // bitonic sort by (price bits, name rank)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < n2; i += FIN_THREADS) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const uint64_t ki = s_key[i], kj = s_key[ixj];
          const uint32_t ii = s_idx[i], ij = s_idx[ixj];
          const bool gt = ki > kj || (ki == kj && ii > ij);
          if (gt == ((i & k) == 0)) {
            s_key[i] = kj;
            s_key[ixj] = ki;
            s_idx[i] = ij;
            s_idx[ixj] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  const uint32_t lim = a.max_types ? min(n, (uint32_t)a.max_types) : n;
  for (uint32_t i = threadIdx.x; i < lim; i += FIN_THREADS)
    a.out_options[(size_t)nc * a.opt_stride + i] = s_idx[i] & 4095u;
  if (threadIdx.x == 0) {
    a.out_n_remaining[nc] = n;
    a.out_n_options[nc] = lim;
  }
}

#endif  // KP_TU & 1
#if KP_TU & 2
// ------------------------------------------------------------------------------------------------
// feasibility_kernel: CompatibleAvailableFilter, one query row per wave, lane = type.
// ------------------------------------------------------------------------------------------------
#define FEAS_WAVES 8
#define FEAS_NT 8  // 64-type tiles per lane batch (measured: 4 and 16 are slower)
#ifndef FEAS_MAX_BLOCKS
#define FEAS_MAX_BLOCKS 65536
#endif
// One wave per query row: the row's requirement set is decoded once (allowed value words, negative-operator
// keys, compatible offering classes), then the lane evaluates its types t = tile*64 + lane of FEAS_NT tiles at
// once. Every catalogue gather of one step (a key's codes, a resource's allocatable, a class's prices) is one
// batch of FEAS_NT independent loads, so a row costs ~(keys + resources + classes) L2 round trips instead of
// that many per tile. Outputs: __ballot -> mask word per tile, cheapest price per (row, type) (coalesced).
__global__ __launch_bounds__(FEAS_WAVES * 64) void feasibility_kernel(FeasArgs a) {
  __shared__ DevDict D;
  __shared__ uint64_t s_allowed[FEAS_WAVES][KP_MAX_WORDS];
  block_copy(D, a.dict);
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = LANE;
  // by value: the catalogue pointers live in SGPRs; through a generic reference every field access after an
  // output store was re-read with a FLAT load (which waits for the outstanding stores)
  const DevCatalog Cg = *a.cat;
  const int T = D.T;
  const int tiles = (T + 63) >> 6;
  for (long q = (long)blockIdx.x * FEAS_WAVES + wave; q < a.n_queries; q += (long)gridDim.x * FEAS_WAVES) {
    const KReqs* Q = reinterpret_cast<const KReqs*>(a.q_reqs + (size_t)q * sizeof(KReqs));
    const uint64_t v = lane < D.W ? Q->vals[lane] : 0;
    const int64_t rq_lane = lane < KP_NRES ? a.q_requests[(size_t)q * KP_NRES + lane] : 0;
    ReqView rv;
    rv.present = Q->present;
    rv.compl_ = Q->compl_ & Q->present;
    rv.hgt = Q->hgt;
    rv.hlt = Q->hlt;
    rv.hmin = Q->hmin;
    rv.nz = nz_keys(D, v);
    rv.dne = 0;
    rv.gt = Q->gt;
    rv.lt = Q->lt;
    rv.minv = Q->minv;
    const uint64_t negQ = negop_mask(rv.present, rv.compl_, rv.nz);
    const uint64_t allowed = allowed_word(D, rv, v, vint_global(a.vint));
    const uint64_t cls = allowed_classes<true>(D, Cg.cls, rv, allowed, negQ);
    if (a.out_classes && lane == 0) a.out_classes[q] = cls;
    s_allowed[wave][lane] = allowed;
    const uint32_t rmask = (uint32_t)__ballot(rq_lane > 0);
    wave_sync();
    const uint64_t keys0 = rv.present & D.catalog_keys;
    for (int c0 = 0; c0 < tiles; c0 += FEAS_NT) {
      int tt[FEAS_NT];
      uint32_t alive = 0;
#pragma unroll
      for (int i = 0; i < FEAS_NT; i++) {
        const int t = (c0 + i) * 64 + lane;
        const bool ok = c0 + i < tiles && t < T;
        tt[i] = ok ? t : 0;
        alive |= (uint32_t)ok << i;
      }
      const uint32_t valid = alive;
      // Fits: negative totals never fit (one uniform word per tile)
#pragma unroll
      for (int i = 0; i < FEAS_NT; i++)
        if (c0 + i < tiles && !((Cg.nonneg[c0 + i] >> lane) & 1)) alive &= ~(1u << i);
      // Compatible(q, type, WK) part (a): non-well-known type keys q does not define
      if (a.mode_compatible && (Cg.custom_any & ~rv.present)) {  // skipped when no type has such a key
        uint64_t cn[FEAS_NT];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) cn[i] = Cg.custom_nonneg[tt[i]];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++)
          if (cn[i] & ~rv.present) alive &= ~(1u << i);
      }
      // Intersects over the shared keys: one batch of code gathers per key
      uint64_t keys = keys0;
      while (keys) {
        const int k = __builtin_ctzll(keys);
        keys &= keys - 1;
        const uint16_t* ck = Cg.code + (size_t)k * T;
        uint32_t code[FEAS_NT];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) code[i] = ck[tt[i]];
        uint32_t multi_need = 0;
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) {
          const uint32_t c = code[i];
          bool pass;
          if (c == 0xFFFFu) pass = true;                      // type lacks the key
          else if (c == 0xFFFEu) pass = (negQ >> k) & 1;      // type DoesNotExist: only NotIn/DNE intersect
          else if (c == 0xFFFDu) { pass = true; multi_need |= 1u << i; }
          else pass = (s_allowed[wave][c >> 6] >> (c & 63)) & 1;
          if (!pass) alive &= ~(1u << i);
        }
        multi_need &= alive;
        if (__ballot(multi_need != 0)) {
          const uint64_t aw = s_allowed[wave][D.wofs[k]];
          const uint64_t* mk = Cg.multi + (size_t)k * T;
          uint64_t mv[FEAS_NT];
#pragma unroll
          for (int i = 0; i < FEAS_NT; i++) mv[i] = (multi_need >> i) & 1 ? mk[tt[i]] : ~0ull;
#pragma unroll
          for (int i = 0; i < FEAS_NT; i++)
            if ((aw & mv[i]) == 0) alive &= ~(1u << i);
        }
      }
      // Fits on the requested resources
      uint32_t rm = rmask;
      while (rm) {
        const int r = __builtin_ctz(rm);
        rm &= rm - 1;
        const int64_t need = lane_bcast_i64(rq_lane, r);
        const int64_t* ar = Cg.alloc + (size_t)r * T;
        int64_t al[FEAS_NT];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) al[i] = ar[tt[i]];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++)
          if (need > al[i]) alive &= ~(1u << i);
      }
      // cheapest compatible available offering (per-lane min over the row's classes)
      double cheapest[FEAS_NT];
#pragma unroll
      for (int i = 0; i < FEAS_NT; i++) cheapest[i] = __builtin_huge_val();
      uint64_t m = cls;
      if (Cg.price_sub) {  // one gather: the min over the row's class set is precomputed per subset
        const double* ps = Cg.price_sub + (size_t)cls * T;
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) cheapest[i] = ps[tt[i]];
        m = 0;
      }
      while (m) {
        const int c = __builtin_ctzll(m);
        m &= m - 1;
        const double* pc = Cg.price_cm + (size_t)c * T;
        double p[FEAS_NT];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) p[i] = pc[tt[i]];
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++) cheapest[i] = p[i] < cheapest[i] ? p[i] : cheapest[i];
      }
      uint64_t myword = 0;
#pragma unroll
      for (int i = 0; i < FEAS_NT; i++) {
        const bool keep = ((alive >> i) & 1) && cheapest[i] < __builtin_huge_val();
        const uint64_t bal = __ballot(keep);
        if (lane == i) myword = bal;
      }
      const int nt = min(FEAS_NT, tiles - c0);
      if (lane < nt) a.out_mask[(size_t)q * tiles + c0 + lane] = myword;
      if (a.out_cheapest) {
        double* oc = a.out_cheapest + (size_t)q * a.ch_stride;
#pragma unroll
        for (int i = 0; i < FEAS_NT; i++)
          if ((valid >> i) & 1) oc[tt[i]] = cheapest[i];
      }
    }
    wave_sync();
  }
}

// feasibility_bits_kernel: the same filter, each row evaluated as bitsets over the whole catalogue. One wave per row;
// lane l < TW holds the row's verdict for types 64 l .. 64 l + 63 as one word, built from the catalogue's type-set
// rows (L2-resident): per key, NOKEY | (NotIn/DoesNotExist ? DNE) | the union of TM rows of the key's allowed values
// (for a single-valued key, when fewer, the complement: valued types minus the union over its excluded values);
// Fits as one threshold row per requested resource (fit_mask at the first allocatable >= the request); an available
// compatible offering as the union of the row's classes' offer_avail rows. The mask words are the lanes' words: no
// per-type work. The cheapest compatible available price per type is the row price_sub[cls] of the precomputed
// per-class-subset minima (a row copy, L2 -> HBM), or the min over the classes' price rows when C > KP_SUB_MAX_C.
// The next row's header loads are issued before this row is evaluated.
#define FEASB_WAVES 8
#define FEASB_CP 8    // cheapest-row copy: loads in flight per lane before their stores (measured: 16 is slower)
#define FEASB_MINW 8  // waves per SIMD the register budget must allow (measured: 0.1574 -> 0.1245 ms on 50k rows)
__global__ __launch_bounds__(FEASB_WAVES * 64, FEASB_MINW) void feasibility_bits_kernel(FeasArgs a) {
  __shared__ DevDict D;
  block_copy(D, a.dict);
  __shared__ int64_t s_vint[KP_MAX_BOUND_KEYS * 64];
  __shared__ OfferClass s_cls[KP_MAX_CLASSES];
  const int tid = threadIdx.x;
  constexpr int NT = FEASB_WAVES * 64;
  const DevCatalog Cd = *a.cat;
  const GLB uint64_t* TM = (const GLB uint64_t*)Cd.TM;
  const GLB uint64_t* DNE = (const GLB uint64_t*)Cd.DNE;
  const GLB uint64_t* NOKEY = (const GLB uint64_t*)Cd.NOKEY;
  const GLB uint64_t* fit_mask = (const GLB uint64_t*)Cd.fit_mask;
  const GLB int64_t* fit_vals = (const GLB int64_t*)Cd.fit_vals;
  const GLB int32_t* fit_n = (const GLB int32_t*)Cd.fit_n;
  const GLB uint64_t* offer = (const GLB uint64_t*)Cd.offer_avail;
  const GLB double* price_sub = (const GLB double*)Cd.price_sub;
  const GLB double* price_cm = (const GLB double*)Cd.price_cm;
  const GLB uint64_t* custom = (const GLB uint64_t*)Cd.custom_nonneg;
  __syncthreads();
  const int T = D.T, TW = D.TW, C = D.C;
  for (int i = tid; i < D.KB * 64; i += NT) s_vint[i] = a.vint[i];
  for (int i = tid; i < C; i += NT) s_cls[i] = Cd.cls[i];
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = LANE;
  const bool lw = lane < TW;  // this lane holds a type word
  const uint64_t nonneg = lw ? ((const GLB uint64_t*)Cd.nonneg)[lane] : 0;
  struct RowHdr {
    uint64_t hw, v;
    int64_t rq, gt, lt;
  };
  auto load_row = [&](long q) {
    RowHdr h;
    const GLB KReqs* Q = reinterpret_cast<const GLB KReqs*>((const GLB uint8_t*)a.q_reqs + (size_t)q * sizeof(KReqs));
    h.hw = lane < 6 ? reinterpret_cast<const GLB uint64_t*>(Q)[lane] : 0;
    h.v = lane < D.W ? Q->vals[lane] : 0;
    h.rq = lane < KP_NRES ? ((const GLB int64_t*)a.q_requests)[(size_t)q * KP_NRES + lane] : 0;
    h.gt = lane < KP_MAX_BOUND_KEYS ? Q->gt[lane] : 0;
    h.lt = lane < KP_MAX_BOUND_KEYS ? Q->lt[lane] : 0;
    return h;
  };
  const long q_stride = (long)gridDim.x * FEASB_WAVES;
  long q = (long)blockIdx.x * FEASB_WAVES + wave;
  RowHdr nxt = q < a.n_queries ? load_row(q) : RowHdr{0, 0, 0, 0, 0};
  for (; q < a.n_queries; q += q_stride) {
    const RowHdr cur = nxt;
    if (q + q_stride < a.n_queries) nxt = load_row(q + q_stride);
    const uint64_t v = cur.v;
    ReqView rv;
    rv.present = lane_bcast(cur.hw, 0);
    rv.compl_ = lane_bcast(cur.hw, 1) & rv.present;
    rv.hgt = lane_bcast(cur.hw, 2);
    rv.hlt = lane_bcast(cur.hw, 3);
    rv.hmin = lane_bcast(cur.hw, 4);
    rv.nz = nz_keys(D, v);
    rv.dne = 0;
    rv.gt = rv.lt = nullptr;  // the bounds stay in the lanes (bounds_mask_lanes)
    rv.minv = nullptr;        // minValues plays no part in CompatibleAvailableFilter
    const uint64_t negQ = negop_mask(rv.present, rv.compl_, rv.nz);
    uint64_t allowed;  // allowed_word() with the lane-held bounds
    {
      const uint64_t bk = (rv.hgt | rv.hlt) & rv.present & rv.compl_ & ((1ull << D.KB) - 1);
      const uint64_t bm = bk ? bounds_mask_lanes(D, bk, rv.hgt, rv.hlt, cur.gt, cur.lt, (const int64_t LDS*)s_vint, D.KB,
                                                 (const GLB int64_t*)a.vint)
                             : ~0ull;
      const int k = lane < D.W ? (int)D.wkey[lane] : 0;
      allowed = lane >= D.W ? 0
                : !((rv.present >> k) & 1) ? D.validbits[lane]
                : ((rv.compl_ >> k) & 1)   ? (~v & D.validbits[lane] & bm)
                                            : v;
    }
    const uint64_t cls = allowed_classes<true>(D, (const OfferClass LDS*)s_cls, rv, allowed, negQ);
    if (a.out_classes && lane == 0) a.out_classes[q] = cls;
    // cheapest compatible available offering price per type
    auto cheapest_row = [&]() {
      if (!a.out_cheapest) return;
      GLB double* oc = (GLB double*)a.out_cheapest + (size_t)q * a.ch_stride;
      if (price_sub) {
        // a row copy through range-checked buffer descriptors (num_records = the row's bytes: the hardware drops
        // the tail lanes' accesses), so the loop has no per-element branch: FEASB_CP loads in flight per lane, each
        // store waiting only for its own load (predicated stores compiled to one branch and a full drain each)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(uintptr_t)(price_sub + (size_t)cls * T), 0, T * 8, KP_BUF_DWORD3);
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)oc, 0, T * 8, KP_BUF_DWORD3);
        const bool nt = a.pad_ & 1;
        for (int t0 = 0; t0 < T; t0 += 64 * FEASB_CP) {
          const int vo = (t0 + lane) * 8;  // the whole offset in the VGPR + immediate (the range-checked part)
          u32x2 vv[FEASB_CP];
#pragma unroll
          for (int i = 0; i < FEASB_CP; i++) vv[i] = __builtin_amdgcn_raw_buffer_load_b64(rs, vo + i * 512, 0, 0);
          if (nt) {
#pragma unroll
            for (int i = 0; i < FEASB_CP; i++) __builtin_amdgcn_raw_buffer_store_b64(vv[i], ro, vo + i * 512, 0, 2);
          } else {
#pragma unroll
            for (int i = 0; i < FEASB_CP; i++) __builtin_amdgcn_raw_buffer_store_b64(vv[i], ro, vo + i * 512, 0, 0);
          }
        }
      } else {
        for (int t = lane; t < T; t += 64) {
          double ch = __builtin_huge_val();
          for (uint64_t m = cls; m; m &= m - 1) ch = fmin(ch, price_cm[(size_t)__builtin_ctzll(m) * T + t]);
          oc[t] = ch;
        }
      }
    };
    const uint32_t rmask = (uint32_t)__ballot(cur.rq > 0);
    uint64_t pass = nonneg;
    // Compatible(q, type, WK) part (a): types with a non-well-known key q does not define (rare: per-type loads)
    if (a.mode_compatible && (Cd.custom_any & ~rv.present) && __ballot(lw && pass)) {
      uint64_t keep = 0;
      if (lw)
        for (uint64_t m = pass; m; m &= m - 1) {
          const int b = __builtin_ctzll(m);
          if (!(custom[lane * 64 + b] & ~rv.present)) keep |= 1ull << b;
        }
      pass = keep;
    }
    // Intersects over the shared keys, one key's type set at a time
    for (uint64_t km = rv.present & D.catalog_keys; km; km &= km - 1) {
      const int k = __builtin_ctzll(km);
      uint64_t acc = lw ? NOKEY[(size_t)k * TW + lane] | (((negQ >> k) & 1) ? DNE[(size_t)k * TW + lane] : 0) : 0;
      // the key's value words: allowed (A) and excluded (E) value bits
      int nA = 0, nE = 0;
      uint64_t wm = 1ull << k;
      if ((D.multiword >> k) & 1) wm |= D.ovfmask[k];
      for (uint64_t m = wm; m; m &= m - 1) {
        const int w = __builtin_ctzll(m);
        const uint64_t aw = lane_bcast(allowed, w);
        nA += __builtin_popcountll(aw & D.validbits[w]);
        nE += __builtin_popcountll(~aw & D.validbits[w]);
      }
      const bool compl_walk = ((D.single_valued >> k) & 1) && nE < nA;
      uint64_t u = 0;
      for (uint64_t m = wm; m; m &= m - 1) {
        const int w = __builtin_ctzll(m);
        const uint64_t aw = lane_bcast(allowed, w);
        for (uint64_t bits = (compl_walk ? ~aw : aw) & D.validbits[w]; bits; bits &= bits - 1)
          u |= lw ? TM[(size_t)(w * 64 + __builtin_ctzll(bits)) * TW + lane] : 0;
      }
      if (compl_walk) {  // valued types (single-valued key: not NOKEY, not DNE) outside the excluded values' union
        const uint64_t nk = lw ? NOKEY[(size_t)k * TW + lane] | DNE[(size_t)k * TW + lane] : ~0ull;
        u = ~nk & ~u;
      }
      pass &= acc | u;
    }
    // Fits on the requested resources: the threshold row of the first allocatable >= the request
    for (uint32_t rm = rmask; rm; rm &= rm - 1) {
      const int r = __builtin_ctz(rm);
      const int64_t need = lane_bcast_i64(cur.rq, r);
      uint64_t nb = 0;
      const int n = fit_n[r];
      const int j = wave_lower_bound(fit_vals + (size_t)r * T, n, need, &nb);
      pass &= (j < n && lw) ? fit_mask[((size_t)r * T + j) * TW + lane] : 0;
    }
    // an available offering of a compatible class
    uint64_t av = 0;
    for (uint64_t m = cls; m; m &= m - 1) av |= lw ? offer[(size_t)__builtin_ctzll(m) * TW + lane] : 0;
    pass &= av;
    if (lw) ((GLB uint64_t*)a.out_mask)[(size_t)q * TW + lane] = pass;
    cheapest_row();
  }
}

// feasibility_quad_kernel: feasibility_bits_kernel's filter for catalogues of <= 1024 types (TW <= 16), four rows per
// wave. Each row is decoded by the whole wave as there (requirement words, bounds, Offerings classes: the lane layout
// needs all 64 lanes) and staged in LDS; then the type-set work runs once for the four rows at a time: lane group g
// (lanes 16 g .. 16 g + 15) evaluates row g, lane l of the group holding type word l. One load instruction gathers
// the four rows' words, so the per-row cost of the key walks, the Fits lower bounds (16-ary, in the group) and the
// offering rows drops by up to four; the groups' loops diverge only where the rows do. The rows' cheapest-price
// copies follow, one row at a time over the whole wave. Every type-set load is a buffer load whose inactive lanes
// carry an out-of-range offset (they read 0): no load sits in a branch.
#define FEASQ_OOB 0x7ffffff0  // a buffer offset past every record count (reads 0)
#ifndef FEASQ_EW
#define FEASQ_EW 7      // eval waves per block (the other FEASB_WAVES - FEASQ_EW copy the cheapest-price rows)
#endif
#ifndef FEASQ_ROWS
#define FEASQ_ROWS 28   // rows per block (one quad per eval wave)
#endif
#ifndef FEASQ_B128
#define FEASQ_B128 1    // copy waves move 16 bytes per lane and instruction (0: 8)
#endif
#ifndef FEASQ_SKIP_EVAL
#define FEASQ_SKIP_EVAL 0  // measurement only: decode + copies, no type-set work (wrong masks)
#endif
#ifndef FEASQ_MINW
#define FEASQ_MINW 6  // waves per SIMD the quad kernel's register budget targets (8: 9 VGPRs spilled; 6: none, -4..6 %)
#endif
static_assert(KP_DIAG_BUILD || (FASTLANE == 1 && FL_NOTIME == 1 && FT_FINE == 0 && FAST_SCAN_MAX == 512 &&
                                 FAST_CHK_LIVE == 8 && FAST_EX_ROUNDS == 8 && FAST_CONT == 1 && SORT_DIAG == 0 && EX_DIAG == 0 && FX_DIAG == 0 && FEAS_MAX_BLOCKS == 65536 &&
                                 FEASQ_EW == 7 && FEASQ_ROWS == 28 && FEASQ_B128 == 1 && FEASQ_SKIP_EVAL == 0 && FL_SKIP == 0 &&
                                 FEASQ_MINW == 6),
              "the production build carries the production values of every measurement knob");
// EW eval waves (4 * EW rows per block); FEASB_WAVES - EW copy waves write the cheapest-price rows. Without price rows
// (mask only, or the compact result) every wave evaluates: EW = FEASB_WAVES.
template <int EW>
__global__ __launch_bounds__(FEASB_WAVES * 64, FEASQ_MINW) void feasibility_quad_kernel(FeasArgs a) {
  constexpr int ROWS = 4 * EW;
  __shared__ DevDict D;
  __shared__ int64_t s_vint[KP_MAX_BOUND_KEYS * 64];
  __shared__ OfferClass s_cls[KP_MAX_CLASSES];
  __shared__ int32_t s_fitn[KP_NRES];
  __shared__ uint64_t s_allow[FEASB_WAVES][4][KP_MAX_WORDS];  // each row's allowed value words
  __shared__ uint64_t s_rowh[FEASB_WAVES][4][4];              // keys, negQ, classes, requested-resource mask
  __shared__ int64_t s_rq[FEASB_WAVES][4][KP_NRES];           // requests
  __shared__ uint64_t s_pass0[FEASB_WAVES][4][16];            // the type words before the AND chain
  __shared__ uint64_t s_rcls[ROWS];                      // each row's offering classes, for the copy waves
  __shared__ int32_t s_ready[ROWS];                      // ... once published
  for (int i = threadIdx.x; i < ROWS; i += FEASB_WAVES * 64) s_ready[i] = 0;
  block_copy(D, a.dict);
  const int tid = threadIdx.x;
  constexpr int NT = FEASB_WAVES * 64;
  const DevCatalog Cd = *a.cat;
  const GLB double* price_sub = (const GLB double*)Cd.price_sub;
  const GLB double* price_cm = (const GLB double*)Cd.price_cm;
  const GLB uint64_t* custom = (const GLB uint64_t*)Cd.custom_nonneg;
  __syncthreads();
  const int T = D.T, TW = D.TW, C = D.C;
  for (int i = tid; i < D.KB * 64; i += NT) s_vint[i] = a.vint[i];
  for (int i = tid; i < C; i += NT) s_cls[i] = Cd.cls[i];
  for (int i = tid; i < KP_NRES; i += NT) s_fitn[i] = Cd.fit_n[i];
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = LANE;
  const bool lw = lane < TW;
  const uint64_t nonneg = lw ? ((const GLB uint64_t*)Cd.nonneg)[lane] : 0;
  const int row8 = TW * 8;
  const __amdgpu_buffer_rsrc_t r_tm = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.TM, 0, D.W * 64 * row8, KP_BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t r_nk = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.NOKEY, 0, D.K * row8, KP_BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t r_dne = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.DNE, 0, D.K * row8, KP_BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t r_fv = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.fit_vals, 0, KP_NRES * T * 8, KP_BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t r_fm = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.fit_mask, 0, KP_NRES * T * row8, KP_BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t r_of = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)Cd.offer_avail, 0, C * row8, KP_BUF_DWORD3);
  auto ld64 = [](const __amdgpu_buffer_rsrc_t& r, int off) -> uint64_t {
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return ((uint64_t)x.y << 32) | x.x;
  };
  struct RowHdr {
    uint64_t hw, v;
    int64_t rq, gt, lt;
  };
  auto load_row = [&](long q) {
    RowHdr h;
    const GLB KReqs* Q = reinterpret_cast<const GLB KReqs*>((const GLB uint8_t*)a.q_reqs + (size_t)q * sizeof(KReqs));
    h.hw = lane < 6 ? reinterpret_cast<const GLB uint64_t*>(Q)[lane] : 0;
    h.v = lane < D.W ? Q->vals[lane] : 0;
    h.rq = lane < KP_NRES ? ((const GLB int64_t*)a.q_requests)[(size_t)q * KP_NRES + lane] : 0;
    h.gt = lane < KP_MAX_BOUND_KEYS ? Q->gt[lane] : 0;
    h.lt = lane < KP_MAX_BOUND_KEYS ? Q->lt[lane] : 0;
    return h;
  };
  // the block's rows: [row0, row1), ROWS per block; eval waves take its quads in turn, copy waves its rows
  const long n = a.n_queries;
  const long row0 = (long)blockIdx.x * ROWS, row1 = min(row0 + ROWS, n);
  if (wave >= EW) {  // ---- a copy wave: each row's cheapest-price row once its eval wave published the classes
    if (a.out_cheapest) {
      // items = (row, half): T <= 1024, so a row is two 512-type halves (a short one reads 0 / drops its stores). The
      // next item's loads are issued before this item's stores: the in-order vector-memory counter then waits for a
      // load without waiting for the stores issued just before it
      const int ncw = FEASB_WAVES - EW > 0 ? FEASB_WAVES - EW : 1, cw = wave - EW;  // (EW == FEASB_WAVES: no copy wave)
      const long nrows = row1 - row0;
      const int nitems = nrows > cw ? 2 * (int)((nrows - cw + ncw - 1) / ncw) : 0;
      auto row_of = [&](int it) { return row0 + cw + (long)(it >> 1) * ncw; };
#if FEASQ_B128
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      auto issue = [&](int it, u32x4 (&v)[8]) {
        const long q = row_of(it);
        const int j = (int)(q - row0);
        while (__hip_atomic_load(&s_ready[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(2);
        asm volatile("" ::: "memory");
        const uint64_t cls = s_rcls[j];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(uintptr_t)(price_sub + (size_t)cls * T), 0, T * 8, KP_BUF_DWORD3);
        const int vo = ((it & 1) * 512 + lane * 2) * 8;
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + i * 1024, 0, 0);
      };
      auto store = [&](int it, const u32x4 (&v)[8]) {
        GLB double* oc = (GLB double*)a.out_cheapest + (size_t)row_of(it) * a.ch_stride;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)oc, 0, T * 8, KP_BUF_DWORD3);
        const int vo = ((it & 1) * 512 + lane * 2) * 8;
#pragma unroll
        for (int i = 0; i < 4; i++) __builtin_amdgcn_raw_buffer_store_b128(v[i], ro, vo + i * 1024, 0, 2);
      };
      typedef u32x4 CpT;
#else
      typedef u32x2 CpT;
      auto issue = [&](int it, u32x2 (&v)[8]) {
        const long q = row_of(it);
        const int j = (int)(q - row0);
        while (__hip_atomic_load(&s_ready[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(2);
        asm volatile("" ::: "memory");  // (the classes are read after the flag: LDS requests complete in order)
        const uint64_t cls = s_rcls[j];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(uintptr_t)(price_sub + (size_t)cls * T), 0, T * 8, KP_BUF_DWORD3);
        const int vo = ((it & 1) * 512 + lane) * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b64(rs, vo + i * 512, 0, 0);
      };
      auto store = [&](int it, const u32x2 (&v)[8]) {
        GLB double* oc = (GLB double*)a.out_cheapest + (size_t)row_of(it) * a.ch_stride;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)oc, 0, T * 8, KP_BUF_DWORD3);
        const int vo = ((it & 1) * 512 + lane) * 8;
        if (a.pad_ & 1) {
#pragma unroll
          for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b64(v[i], ro, vo + i * 512, 0, 2);
        } else {
#pragma unroll
          for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b64(v[i], ro, vo + i * 512, 0, 0);
        }
      };
#endif
      if (price_sub) {
        CpT P[8], Q[8];
        if (nitems) issue(0, P);
        for (int it = 0; it < nitems; it += 2) {  // (nitems is even)
          issue(it + 1, Q);
          store(it, P);
          if (it + 2 < nitems) issue(it + 2, P);
          store(it + 1, Q);
        }
      } else {
        for (long q = row0 + cw; q < row1; q += ncw) {
          const int j = (int)(q - row0);
          while (__hip_atomic_load(&s_ready[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(2);
        asm volatile("" ::: "memory");  // (the classes are read after the flag: LDS requests complete in order)
          const uint64_t cls = s_rcls[j];
          GLB double* oc = (GLB double*)a.out_cheapest + (size_t)q * a.ch_stride;
          for (int t = lane; t < T; t += 64) {
            double ch = __builtin_huge_val();
            for (uint64_t m = cls; m; m &= m - 1) ch = fmin(ch, price_cm[(size_t)__builtin_ctzll(m) * T + t]);
            oc[t] = ch;
          }
        }
      }
    }
    return;
  }
  const long quads = (row1 - row0 + 3) / 4;
  long qi = wave;
  RowHdr nxt = qi < quads ? load_row(row0 + 4 * qi) : RowHdr{0, 0, 0, 0, 0};
  for (; qi < quads; qi += EW) {
    const long qd_base = row0 + 4 * qi;
    // ---- phase 1: decode the four rows (the next row's header loads in flight meanwhile)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const long q = qd_base + r;
      const long qn = r < 3 ? q + 1 : qd_base + 4 * EW;
      const RowHdr cur = nxt;
      if (qn < row1) nxt = load_row(qn);
      if (q >= row1) {  // past the block's last row: an empty group
        if (lane < 4) s_rowh[wave][r][lane] = 0;
        if (lane < 16) s_pass0[wave][r][lane] = 0;
        continue;
      }
      const uint64_t v = cur.v;
      ReqView rv;
      rv.present = lane_bcast(cur.hw, 0);
      rv.compl_ = lane_bcast(cur.hw, 1) & rv.present;
      rv.hgt = lane_bcast(cur.hw, 2);
      rv.hlt = lane_bcast(cur.hw, 3);
      rv.hmin = lane_bcast(cur.hw, 4);
      rv.nz = nz_keys(D, v);
      rv.dne = 0;
      rv.gt = rv.lt = nullptr;
      rv.minv = nullptr;
      const uint64_t negQ = negop_mask(rv.present, rv.compl_, rv.nz);
      uint64_t allowed;
      {
        const uint64_t bk = (rv.hgt | rv.hlt) & rv.present & rv.compl_ & ((1ull << D.KB) - 1);
        const uint64_t bm = bk ? bounds_mask_lanes(D, bk, rv.hgt, rv.hlt, cur.gt, cur.lt, (const int64_t LDS*)s_vint, D.KB,
                                                   (const GLB int64_t*)a.vint)
                               : ~0ull;
        const int k = lane < D.W ? (int)D.wkey[lane] : 0;
        allowed = lane >= D.W ? 0
                  : !((rv.present >> k) & 1) ? D.validbits[lane]
                  : ((rv.compl_ >> k) & 1)   ? (~v & D.validbits[lane] & bm)
                                              : v;
      }
      const uint64_t cls = allowed_classes<true>(D, (const OfferClass LDS*)s_cls, rv, allowed, negQ);
      if (lane == 0 && a.out_classes) a.out_classes[q] = cls;  // the compact result
      if (lane == 0) {  // published to the copy waves (LDS writes complete in order: the classes before the flag;
                        // a relaxed workgroup-scope flag keeps this wave's vector-memory queue undrained)
        s_rcls[q - row0] = cls;
        asm volatile("" ::: "memory");
        __hip_atomic_store(&s_ready[q - row0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      uint64_t pass = nonneg;
      // Compatible(q, type, WK) part (a): types with a non-well-known key q does not define (rare: per-type loads)
      if (a.mode_compatible && (Cd.custom_any & ~rv.present) && __ballot(lw && pass)) {
        uint64_t keep = 0;
        if (lw)
          for (uint64_t m = pass; m; m &= m - 1) {
            const int b = __builtin_ctzll(m);
            if (!(custom[lane * 64 + b] & ~rv.present)) keep |= 1ull << b;
          }
        pass = keep;
      }
      s_allow[wave][r][lane] = allowed;
      if (lane < 16) s_pass0[wave][r][lane] = pass;
      if (lane < KP_NRES) s_rq[wave][r][lane] = cur.rq;
      const uint64_t rmask = (uint64_t)(uint32_t)__ballot(cur.rq > 0);
      if (lane == 0) {
        s_rowh[wave][r][0] = rv.present & D.catalog_keys;
        s_rowh[wave][r][1] = negQ;
        s_rowh[wave][r][2] = cls;
        s_rowh[wave][r][3] = rmask;
      }
    }
    wave_sync();
    // ---- phase 2: the four rows' type-set work, lane group g on row g
    if (!FEASQ_SKIP_EVAL) {
      const int g = lane >> 4, l = lane & 15;
      const bool gl = l < TW;
      const int lo8 = l * 8;
      const long q = qd_base + g;
      const uint64_t keys = s_rowh[wave][g][0], negQ = s_rowh[wave][g][1], cls = s_rowh[wave][g][2];
      const uint32_t rmask = (uint32_t)s_rowh[wave][g][3];
      uint64_t pass = gl ? s_pass0[wave][g][l] : 0;
      auto off = [&](int row) { return gl ? row * row8 + lo8 : FEASQ_OOB; };
      // Intersects over the shared keys (as feasibility_bits_kernel; a single-valued key with fewer excluded than
      // allowed values: the complement of (negQ ? 0 : DNE) | the excluded values' TM rows, NOKEY, DNE and the TM
      // rows being disjoint by construction)
      for (uint64_t km = keys; km; km &= km - 1) {
        const int k = __builtin_ctzll(km);
        const bool nq = (negQ >> k) & 1;
        uint64_t wm = 1ull << k;
        if ((D.multiword >> k) & 1) wm |= D.ovfmask[k];
        int nA = 0, nE = 0;
        for (uint64_t m = wm; m; m &= m - 1) {
          const int w = __builtin_ctzll(m);
          const uint64_t aw = s_allow[wave][g][w], vb = D.validbits[w];
          nA += __builtin_popcountll(aw & vb);
          nE += __builtin_popcountll(~aw & vb);
        }
        const bool compl_walk = ((D.single_valued >> k) & 1) && nE < nA;
        uint64_t u = compl_walk ? (nq ? 0 : ld64(r_dne, off(k))) : (ld64(r_nk, off(k)) | (nq ? ld64(r_dne, off(k)) : 0));
        for (uint64_t m = wm; m; m &= m - 1) {
          const int w = __builtin_ctzll(m);
          const uint64_t aw = s_allow[wave][g][w];
          for (uint64_t bits = (compl_walk ? ~aw : aw) & D.validbits[w]; bits; bits &= bits - 1)
            u |= ld64(r_tm, off(w * 64 + __builtin_ctzll(bits)));
        }
        pass &= compl_walk ? ~u : u;
      }
      // Fits: the threshold row of the first allocatable >= the request (a 16-ary lower bound in the group)
      for (uint32_t rm = rmask; rm; rm &= rm - 1) {
        const int r = __builtin_ctz(rm);
        const int64_t need = s_rq[wave][g][r];
        const int nr = s_fitn[r];
        int lo = 0, hi = nr;
        while (lo < hi) {
          const int span = hi - lo, step = span <= 16 ? 1 : (span + 15) / 16, idx = lo + l * step;
          const int64_t x = (int64_t)ld64(r_fv, idx < hi ? (r * T + idx) * 8 : FEASQ_OOB);
          const uint32_t gb = (uint32_t)(__ballot(idx < hi && x >= need) >> (16 * g)) & 0xffffu;
          if (span <= 16) {
            lo = hi = gb ? lo + __builtin_ctz(gb) : hi;
          } else if (!gb) {
            lo = lo + min(15, (hi - 1 - lo) / step) * step + 1;
          } else {
            const int f = __builtin_ctz(gb);
            if (f == 0) {
              hi = lo;
            } else {
              const int nlo = lo + (f - 1) * step + 1;
              hi = lo + f * step;
              lo = nlo;
            }
          }
        }
        pass &= ld64(r_fm, lo < nr ? off(r * T + lo) : FEASQ_OOB);  // no threshold: 0
      }
      // an available offering of a compatible class
      uint64_t av = 0;
      for (uint64_t m = cls; m; m &= m - 1) av |= ld64(r_of, off(__builtin_ctzll(m)));
      pass &= av;
      if (gl && q < row1) ((GLB uint64_t*)a.out_mask)[(size_t)q * TW + l] = pass;
    }
    wave_sync();  // (phase 1 of the next quad rewrites this wave's LDS rows)
  }
}

#endif  // KP_TU & 2
#if KP_TU & 1
// ------------------------------------------------------------------------------------------------
// launch_kernel: instance.DefaultProvider.Create's launch-side selection (R:pkg/providers/instance/instance.go:
// 117-125, 242-270, 336-355, 392-439, 504-518), one wave per NodeClaim request. Lane = list entry: the
// CompatibleAvailable test and the cheapest compatible available prices per capacity type are one pass over the
// list; the exotic and spot filters are wave reductions + an ordered compaction in LDS; Truncate is a bitonic sort
// by (price, name) of the survivors; overrides are a wave prefix sum over the truncated entries.
// ------------------------------------------------------------------------------------------------
#define LAUNCH_WAVES 4
struct LaunchWaveLds {
  uint64_t allowed[KP_MAX_WORDS];
  uint64_t key[LAUNCH_CAP];  // cheapest available compatible price (bits; non-negative doubles order as integers)
  uint32_t val[LAUNCH_CAP];  // name rank << 12 | type, bit 31: exotic
  uint64_t xm[KP_MAX_TYPE_WORDS];
  uint32_t scratch[2 * KP_MAX_WORDS];
};
#define LV_ORDER(v) ((v) & 0x00FFFFFFu)

// ordered compaction of the m entries in L.key/L.val keeping those whose keep() is true; returns the new count
template <class Keep>
__device__ int launch_compact(LaunchWaveLds& L, int m, Keep keep) {
  const int lane = LANE;
  int out = 0;
  for (int base = 0; base < m; base += 64) {
    const int i = base + lane;
    uint64_t k = 0;
    uint32_t v = 0;
    bool kp = false;
    if (i < m) {
      k = L.key[i];
      v = L.val[i];
      kp = keep(k, v);
    }
    const uint64_t bal = __ballot(kp);
    wave_sync();
    if (kp) {
      const int pos = out + __builtin_popcountll(bal & ((1ull << lane) - 1));
      L.key[pos] = k;
      L.val[pos] = v;
    }
    out += __builtin_popcountll(bal);
    wave_sync();
  }
  return out;
}

__global__ __launch_bounds__(LAUNCH_WAVES * 64) void launch_kernel(LaunchArgs a) {
  __shared__ DevDict D;
  __shared__ LaunchWaveLds Wl[LAUNCH_WAVES];
  block_copy(D, a.dict);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = LANE;
  const DevCatalog& Cg = *a.cat;
  LaunchWaveLds& L = Wl[wave];
  const double INF = __builtin_huge_val();
  uint64_t evals = 0, bytes = 0;
  for (long q = (long)blockIdx.x * LAUNCH_WAVES + wave; q < a.n; q += (long)gridDim.x * LAUNCH_WAVES) {
    const KReqs* Q = reinterpret_cast<const KReqs*>(a.q_reqs + (size_t)q * sizeof(KReqs));
    const uint64_t v = lane < D.W ? Q->vals[lane] : 0;
    ReqView rv;
    rv.present = Q->present;
    rv.compl_ = Q->compl_ & Q->present;
    rv.hgt = Q->hgt;
    rv.hlt = Q->hlt;
    rv.hmin = Q->hmin;
    rv.nz = nz_keys(D, v);
    rv.dne = 0;
    rv.gt = Q->gt;
    rv.lt = Q->lt;
    rv.minv = Q->minv;
    const uint64_t negQ = negop_mask(rv.present, rv.compl_, rv.nz);
    const uint64_t allowed = allowed_word(D, rv, v, vint_global(a.vint));
    const uint64_t cls = allowed_classes<true>(D, Cg.cls, rv, allowed, negQ);
    // the same with the capacity-type key opened: getCapacityType / getOverrides pin it to one value
    const bool ctw = a.ct_key >= 0 && lane < D.W && D.wkey[lane] == a.ct_key;
    const uint64_t cls_noct = allowed_classes<true>(D, Cg.cls, rv, ctw ? D.validbits[lane] : allowed, negQ);
    L.allowed[lane] = allowed;
    const int64_t rq_lane = lane < KP_NRES ? a.q_requests[(size_t)q * KP_NRES + lane] : 0;
    const uint32_t rmask = (uint32_t)__ballot(rq_lane > 0);
    const bool hasMin = (rv.hmin & rv.present) != 0;
    // Requirements.Get(capacity-type).Has(x): an absent key is Exists
    const bool ct_present = a.ct_key >= 0 && ((rv.present >> a.ct_key) & 1);
    const bool ct_compl = ct_present && ((rv.compl_ >> a.ct_key) & 1);
    const bool has_spot = a.spot_bit >= 0 ? bit_of(allowed, a.spot_bit) : (!ct_present || ct_compl);
    const bool has_od = a.od_bit >= 0 ? bit_of(allowed, a.od_bit) : (!ct_present || ct_compl);
    wave_sync();
    const int lb = (int)a.list_off[q], ln = (int)(a.list_off[q + 1] - lb);
    const uint64_t keys0 = rv.present & D.catalog_keys;
    LaunchOut res;
    res.status = KP_LAUNCH_OK;
    res.capacity_type = 0;
    res.n_types = 0;
    res.n_overrides = 0;
    res.failed_filter = -1;
    res.rejected_exotic = 0;
    res.rejected_spot = 0;
    res.od_fallback_warning = 0;
    res.reservation_type = -1;
    res.rejected_reservation = 0;
    res.pad_ = 0;
    // ---- CompatibleAvailableFilter (R:filter.go:51-63) -----------------------------------------------
    int m = 0, n_generic = 0;
    for (int base = 0; base < ln; base += 64) {
      const int i = base + lane;
      bool keep = false, exo = false;
      double cheapest = INF;
      int t = 0;
      if (i < ln) {
        t = (int)a.list[lb + i];
        keep = true;
        if (Cg.custom_nonneg[t] & ~rv.present) keep = false;  // Compatible(part a): undefined custom keys
        uint64_t keys = keys0;
        while (keep && keys) {  // Intersects over the keys both define
          const int k = __builtin_ctzll(keys);
          keys &= keys - 1;
          const uint16_t code = Cg.code[(size_t)k * D.T + t];
          if (code == 0xFFFF) continue;
          if (code == 0xFFFE) keep = (negQ >> k) & 1;
          else if (code == 0xFFFD) keep = (L.allowed[D.wofs[k]] & Cg.multi[(size_t)k * D.T + t]) != 0;
          else keep = (L.allowed[code >> 6] >> (code & 63)) & 1;
        }
        if (keep && !((Cg.nonneg[t >> 6] >> (t & 63)) & 1)) keep = false;  // Fits: negative totals never fit
        uint32_t rm = rmask;
        while (keep && rm) {
          const int r = __builtin_ctz(rm);
          rm &= rm - 1;
          if (lane_bcast_i64(rq_lane, r) > Cg.alloc[(size_t)r * D.T + t]) keep = false;
        }
        for (uint64_t mm = cls; mm; mm &= mm - 1) {
          const double p = Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)];
          cheapest = p < cheapest ? p : cheapest;
        }
        if (!(cheapest < INF)) keep = false;
        exo = (a.exotic[t >> 6] >> (t & 63)) & 1;
      }
      const uint64_t bal = __ballot(keep);
      if (keep) {
        const int pos = m + __builtin_popcountll(bal & ((1ull << lane) - 1));
        L.key[pos] = (uint64_t)__double_as_longlong(cheapest);
        L.val[pos] = (Cg.name_rank[t] << 12) | (uint32_t)t | (exo ? 0x80000000u : 0u);
      }
      m += __builtin_popcountll(bal);
      n_generic += __builtin_popcountll(__ballot(keep && !exo));
    }
    evals += ln;
    bytes += (uint64_t)ln * (2 * __builtin_popcountll(keys0) + 8 * __builtin_popcount(rmask) + 8 * __builtin_popcountll(cls) + 16);
    wave_sync();
    res.n_compatible = (uint32_t)m;
    if (m == 0) {
      res.status = KP_LAUNCH_INSUFFICIENT_CAPACITY;
      res.failed_filter = KP_FILTER_COMPATIBLE_AVAILABLE;
    }
    // ---- CapacityReservationType / CapacityBlock / ReservedOffering filters (R:filter.go:66-274) -----------
    // Each replaces a kept type's offering slice. As class sets: every remaining type keeps the classes in M
    // (the first two filters narrow all survivors alike), and after the third (rof) type t keeps rof_pick(t).
    uint64_t M = ~0ull;
    bool rof = false;
    const bool has_res = a.res_bit >= 0 ? bit_of(allowed, a.res_bit) : (!ct_present || ct_compl);
    const uint64_t res_cand = cls & a.cls_res;  // compatible reserved classes
    // ReservedOfferingFilter's choice for type t: per zone, the available compatible reserved class in M with the
    // greatest reservation capacity (the first in offering order on ties)
    auto rof_pick = [&](int t) -> uint64_t {
      const uint64_t cand = res_cand & M;
      uint64_t pick = 0;
      for (int j = 0; j < a.MO && cand; j++) {
        const int c = a.ofs_cls[(size_t)t * a.MO + j];
        if (c == 0xFF) break;
        if (!((cand >> c) & 1) || !(Cg.price[(size_t)t * D.C + c] < INF)) continue;
        const int z = Cg.cls[c].zone_bit;
        int cur = -1;
        for (uint64_t pp = pick; pp; pp &= pp - 1)
          if (Cg.cls[__builtin_ctzll(pp)].zone_bit == z) {
            cur = __builtin_ctzll(pp);
            break;
          }
        if (cur < 0) pick |= 1ull << c;
        else if (a.rcap[(size_t)t * D.C + c] > a.rcap[(size_t)t * D.C + cur]) pick = (pick & ~(1ull << cur)) | (1ull << c);
      }
      return pick;
    };
    auto om_of = [&](int t) -> uint64_t { return rof ? rof_pick(t) : M; };
    if (m && has_res) {  // (no compatible reserved class: CapacityReservationType is a no-op, CapacityBlock may still apply)
      // CapacityReservationTypeFilter (R:filter.go:80-144): the partition with the cheapest available compatible
      // reserved offering (ties: default before capacity-block)
      double pmin[2] = {INF, INF};
      for (int i = lane; i < m; i += 64) {
        const int t = (int)(L.val[i] & 4095u);
        for (uint64_t mm = res_cand & (a.cls_rt0 | a.cls_rt1); mm; mm &= mm - 1) {
          const int c = __builtin_ctzll(mm);
          const double p = Cg.price[(size_t)t * D.C + c];
          const int k = ((a.cls_rt1 >> c) & 1) ? 1 : 0;
          pmin[k] = p < pmin[k] ? p : pmin[k];
        }
      }
      for (int o = 32; o >= 1; o >>= 1)
        for (int k = 0; k < 2; k++) {
          const double w = __shfl_xor(pmin[k], o, 64);
          pmin[k] = w < pmin[k] ? w : pmin[k];
        }
      const uint64_t selm = res_cand & (pmin[1] < pmin[0] ? a.cls_rt1 : a.cls_rt0);
      auto in_part = [&](int t) {
        for (uint64_t mm = selm; mm; mm &= mm - 1)
          if (Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)] < INF) return true;
        return false;
      };
      if (pmin[0] < INF || pmin[1] < INF) {  // the selected partition has types
        const int m0 = m;
        m = launch_compact(L, m, [&](uint64_t, uint32_t vv) { return in_part((int)(vv & 4095u)); });
        M = a.cls_res & (pmin[1] < pmin[0] ? a.cls_rt1 : a.cls_rt0);
        res.rejected_reservation += (uint32_t)(m0 - m);
      }
      // CapacityBlockFilter (R:filter.go:160-225): when the first offering of the first type is a capacity block,
      // keep the one type whose cheapest capacity-block offering (any availability) is the cheapest
      bool should = false;
      {
        const int t0 = (int)(L.val[0] & 4095u);
        for (int j = 0; j < a.MO; j++) {
          const int c = a.ofs_cls[(size_t)t0 * a.MO + j];
          if (c == 0xFF) break;
          if ((M >> c) & 1) {
            should = (a.cls_rt1 >> c) & 1;
            break;
          }
        }
      }
      if (should) {
        const uint64_t cb = M & a.cls_res & a.cls_rt1;
        double best_p = INF;
        int best_i = -1, best_c = -1;
        for (int base = 0; base < m; base += 64) {
          const int i = base + lane;
          double p = INF;
          int sc = -1;
          if (i < m) {
            const int t = (int)(L.val[i] & 4095u);
            for (int j = 0; j < a.MO; j++) {
              const int c = a.ofs_cls[(size_t)t * a.MO + j];
              if (c == 0xFF) break;
              if (!((cb >> c) & 1)) continue;
              const double pc = a.price_all[(size_t)t * D.C + c];
              if (sc < 0 || pc < p) {
                p = pc;
                sc = c;
              }
            }
          }
          // first entry with the smallest price in this chunk
          double wp = sc >= 0 ? p : INF;
          int wi = sc >= 0 ? i : INT32_MAX;
          for (int o = 32; o >= 1; o >>= 1) {
            const double op = __shfl_xor(wp, o, 64);
            const int oi = __shfl_xor(wi, o, 64);
            if (op < wp || (op == wp && oi < wi)) {
              wp = op;
              wi = oi;
            }
          }
          const int wc = __shfl(sc, wi == INT32_MAX ? 0 : (wi & 63), 64);
          if (wi != INT32_MAX && (best_i < 0 || wp < best_p)) {
            best_p = wp;
            best_i = wi;
            best_c = wc;
          }
        }
        if (best_i >= 0) {
          const uint64_t k = L.key[best_i];
          const uint32_t vv = L.val[best_i];
          wave_sync();
          if (lane == 0) {
            L.key[0] = k;
            L.val[0] = vv;
          }
          wave_sync();
          res.rejected_reservation += (uint32_t)(m - 1);
          m = 1;
          M = 1ull << best_c;
        }
      }
      // ReservedOfferingFilter (R:filter.go:241-274): types without an available compatible reserved offering are
      // rejected, unless that rejects all
      int n_keep = 0;
      for (int i = lane; i < m; i += 64) n_keep += rof_pick((int)(L.val[i] & 4095u)) != 0;
      for (int o = 32; o >= 1; o >>= 1) n_keep += __shfl_xor(n_keep, o, 64);
      if (n_keep > 0) {
        const int m0 = m;
        m = launch_compact(L, m, [&](uint64_t, uint32_t vv) { return rof_pick((int)(vv & 4095u)) != 0; });
        rof = true;
        res.rejected_reservation += (uint32_t)(m0 - m);
      }
      if (M != ~0ull || rof) {  // OrderByPrice reads the replaced slices
        for (int i = lane; i < m; i += 64) {
          const int t = (int)(L.val[i] & 4095u);
          double cheapest = INF;
          for (uint64_t mm = cls & om_of(t); mm; mm &= mm - 1) {
            const double p = Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)];
            cheapest = p < cheapest ? p : cheapest;
          }
          L.key[i] = (uint64_t)__double_as_longlong(cheapest);
        }
        wave_sync();
      }
    }
    const bool sliced = M != ~0ull || rof;  // every remaining type holds reserved offerings only
    // ---- ExoticInstanceTypeFilter (R:filter.go:289-314) -------------------------------------------------
    if (m && !hasMin) {
      int ng = 0;  // n_generic of the list the reservation filters left
      for (int i = lane; i < m; i += 64) ng += !(L.val[i] & 0x80000000u);
      for (int o = 32; o >= 1; o >>= 1) ng += __shfl_xor(ng, o, 64);
      n_generic = ng;
    }
    if (m && !hasMin && n_generic > 0 && n_generic < m) {
      res.rejected_exotic = (uint32_t)(m - n_generic);
      m = launch_compact(L, m, [](uint64_t, uint32_t vv) { return !(vv & 0x80000000u); });
    }
    // ---- SpotInstanceFilter (R:filter.go:342-382): a no-op over reserved-only slices (no on-demand offering) ----
    if (m && !hasMin && has_od && has_spot && !sliced) {
      double od_min = INF;
      bool any_spot = false;
      for (int base = 0; base < m; base += 64) {
        const int i = base + lane;
        if (i < m) {
          const int t = (int)(L.val[i] & 4095u);
          for (uint64_t mm = cls & a.cls_od; mm; mm &= mm - 1) {
            const double p = Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)];
            od_min = p < od_min ? p : od_min;
          }
          for (uint64_t mm = cls & a.cls_spot; mm; mm &= mm - 1)
            if (Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)] < INF) any_spot = true;
        }
      }
      for (int o = 32; o >= 1; o >>= 1) {
        const double w = __shfl_xor(od_min, o, 64);
        od_min = w < od_min ? w : od_min;
      }
      any_spot = __ballot(any_spot) != 0;
      if (od_min < INF && any_spot) {
        const uint64_t spot_cls = cls & a.cls_spot;
        const int m0 = m;
        m = launch_compact(L, m, [&](uint64_t, uint32_t vv) {
          const int t = (int)(vv & 4095u);
          bool has = false, cheap = false;
          for (uint64_t mm = spot_cls; mm; mm &= mm - 1) {
            const double p = Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)];
            if (p < INF) {
              has = true;
              if (p <= od_min) cheap = true;
            }
          }
          // types with an available compatible reserved offering are always kept (R:filter.go:368-371)
          for (uint64_t mm = res_cand; mm; mm &= mm - 1)
            if (Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)] < INF) return true;
          return cheap || !has;
        });
        res.rejected_spot = (uint32_t)(m0 - m);
        if (m == 0) {
          res.status = KP_LAUNCH_INSUFFICIENT_CAPACITY;
          res.failed_filter = KP_FILTER_SPOT;
        }
      }
    }
    if (m) {
      // ---- Truncate(reqs, max): OrderByPrice (price asc, name asc), cut, SatisfiesMinValues ----------------
      int m2 = 1;
      while (m2 < m) m2 <<= 1;
      for (int i = m + lane; i < m2; i += 64) {
        L.key[i] = ~0ull;
        L.val[i] = 0x00FFFFFFu;
      }
      wave_sync();
      for (int k = 2; k <= m2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = lane; i < m2; i += 64) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const uint64_t ki = L.key[i], kj = L.key[ixj];
              const uint32_t vi = L.val[i], vj = L.val[ixj];
              const bool gt = ki > kj || (ki == kj && LV_ORDER(vi) > LV_ORDER(vj));
              if (gt == ((i & k) == 0)) {
                L.key[i] = kj;
                L.key[ixj] = ki;
                L.val[i] = vj;
                L.val[ixj] = vi;
              }
            }
          }
          wave_sync();
        }
      }
      const int cut = a.max_types ? min(m, a.max_types) : m;
      bool min_ok = true;
      if (hasMin) {
        L.xm[lane] = 0;
        wave_sync();
        for (int i = lane; i < cut; i += 64) {
          const int t = (int)(L.val[i] & 4095u);
          atomicOr((unsigned long long*)&L.xm[t >> 6], 1ull << (t & 63));
        }
        wave_sync();
        min_ok = minvalues_ok(D, Cg.code, Cg.TM, rv.hmin & rv.present, rv.minv, lane < D.TW ? L.xm[lane] : 0,
                              L.scratch);
      }
      if (!min_ok) {
        res.status = KP_LAUNCH_MINVALUES;
      } else {
        // ---- getCapacityType (R:instance.go:504-518) + checkODFallback (:336-355) -------------------------
        // reserved first (R:instance.go:506), then spot, over the (replaced) offering slices
        bool res_ok = false, spot_ok = false;
        for (int i = lane; i < cut; i += 64) {
          const int t = (int)(L.val[i] & 4095u);
          const uint64_t om = om_of(t) & cls_noct;
          if (has_res)
            for (uint64_t mm = om & a.cls_res; mm; mm &= mm - 1)
              if (Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)] < INF) res_ok = true;
          if (has_spot)
            for (uint64_t mm = om & a.cls_spot; mm; mm &= mm - 1)
              if (Cg.price[(size_t)t * D.C + __builtin_ctzll(mm)] < INF) spot_ok = true;
        }
        const bool ct_res = has_res && __ballot(res_ok) != 0;
        const bool ct_spot = !ct_res && has_spot && __ballot(spot_ok) != 0;
        res.capacity_type = ct_res ? 2 : ct_spot ? 1 : 0;
        res.od_fallback_warning = (!ct_res && !ct_spot && has_spot && cut < 5) ? 1 : 0;
        if (ct_res) {  // getCapacityReservationType: the first offering of the first type
          const int t0 = (int)(L.val[0] & 4095u);
          const uint64_t om0 = om_of(t0);
          for (int j = 0; j < a.MO; j++) {
            const int c = a.ofs_cls[(size_t)t0 * a.MO + j];
            if (c == 0xFF) break;
            if ((om0 >> c) & 1) {
              res.reservation_type = ((a.cls_rt0 >> c) & 1) ? 0 : ((a.cls_rt1 >> c) & 1) ? 1 : -1;
              break;
            }
          }
        }
        // ---- getOverrides (R:instance.go:392-439) with the capacity type pinned -----------------------------
        const uint64_t cls3 = cls_noct & (ct_res ? a.cls_res : ct_spot ? a.cls_spot : a.cls_od);
        uint32_t* ot = a.out_types + (size_t)q * a.max_types;
        uint32_t* oo = a.out_overrides + (size_t)q * a.ovr_stride;
        int novr = 0;
        for (int base = 0; base < cut; base += 64) {
          const int i = base + lane;
          int t = 0, cnt = 0;
          uint64_t c3 = 0;
          if (i < cut) {
            t = (int)(L.val[i] & 4095u);
            ot[i] = (uint32_t)t;
            c3 = cls3 & om_of(t);
            for (int j = 0; j < a.MO; j++) {
              const int c = a.ofs_cls[(size_t)t * a.MO + j];
              if (c == 0xFF) break;
              if (((c3 >> c) & 1) && Cg.price[(size_t)t * D.C + c] < INF && a.cls_zone[c] >= 0) cnt++;
            }
          }
          int incl = cnt;  // inclusive wave scan
          for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
          }
          int pos = novr + incl - cnt;
          if (i < cut)
            for (int j = 0; j < a.MO; j++) {
              const int c = a.ofs_cls[(size_t)t * a.MO + j];
              if (c == 0xFF) break;
              if (((c3 >> c) & 1) && Cg.price[(size_t)t * D.C + c] < INF && a.cls_zone[c] >= 0 && pos < (int)a.ovr_stride)
                oo[pos++] = ((uint32_t)t << 8) | (uint32_t)a.cls_zone[c];
            }
          novr += __shfl(incl, 63, 64);
        }
        res.n_types = (uint32_t)cut;
        res.n_overrides = (uint32_t)novr;
      }
    }
    if (lane == 0) a.out[q] = res;
    wave_sync();
  }
  if (lane == 0) {
    atomicAdd((unsigned long long*)&a.stats[0], (unsigned long long)evals);
    atomicAdd((unsigned long long*)&a.stats[1], (unsigned long long)bytes);
  }
}

#include "kp_sim.hip"

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_solve(const SolveArgs& a, int nw, size_t dyn_lds, hipStream_t s) {
  (void)nw;
  // 4 waves (one per SIMD): the per-pod barriers and pre-pass compaction are cheaper than with 8, and 4 candidates per
  // attempt round cover the typical 2-3 attempts per pod (8 waves measured slower)
  if (a.n_groups) hipLaunchKernelGGL((solve_kernel<4, true, false>), dim3(1), dim3(4 * 64), dyn_lds, s, a, nullptr);
  else hipLaunchKernelGGL((solve_kernel<4, false, false>), dim3(1), dim3(4 * 64), dyn_lds, s, a, nullptr);
  return hipGetLastError();
}
hipError_t launch_solve_batch(const SolveArgs& a0, const SolveArgs* dev_args, int n, size_t dyn_lds, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (a0.n_groups) hipLaunchKernelGGL((solve_kernel<4, true, true>), dim3(n), dim3(4 * 64), dyn_lds, s, a0, dev_args);
  else hipLaunchKernelGGL((solve_kernel<4, false, true>), dim3(n), dim3(4 * 64), dyn_lds, s, a0, dev_args);
  return hipGetLastError();
}
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  if (a.n_nc == 0) return hipSuccess;
  hipLaunchKernelGGL((finalize_kernel<false>), dim3(a.n_nc), dim3(FIN_THREADS), 0, s, a, nullptr);
  return hipGetLastError();
}
hipError_t launch_finalize_batch(const FinalizeArgs& a0, const FinalizeArgs* dev_args, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL((finalize_kernel<true>), dim3(n), dim3(FIN_THREADS), 0, s, a0, dev_args);
  return hipGetLastError();
}
// Batched Solves' arenas: every arena [y] = base + y * stride gets the shared pristine block copied to `dst_off` (but
// for one hole the Solve never reads before writing) and its `n_fill` ranges set to their byte (16-byte granules:
// offsets and lengths are multiples of 16).
__global__ __launch_bounds__(256) void batch_init_kernel(BatchInitArgs a) {
  uint8_t* arena = a.base + (size_t)blockIdx.y * a.stride;
  const size_t n16 = a.n_copy / 16;
  const uint4* src = reinterpret_cast<const uint4*>(a.pristine);
  uint4* dst = reinterpret_cast<uint4*>(arena + a.dst_off);
  const size_t s0 = a.skip_off / 16, s1 = (a.skip_off + a.skip_len) / 16;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    if (i < s0 || i >= s1) dst[i] = src[i];
  for (int f = 0; f < a.n_fill; f++) {
    const uint32_t b = a.fill_byte[f];
    const uint4 v = make_uint4(b * 0x01010101u, b * 0x01010101u, b * 0x01010101u, b * 0x01010101u);
    uint4* d = reinterpret_cast<uint4*>(arena + a.fill_off[f]);
    const size_t m = a.fill_len[f] / 16;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (size_t)gridDim.x * 256) d[i] = v;
  }
}
hipError_t launch_batch_init(const BatchInitArgs& a, int n_arenas, hipStream_t s) {
  if (n_arenas <= 0) return hipSuccess;
  hipLaunchKernelGGL(batch_init_kernel, dim3(64, n_arenas), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_launch(const LaunchArgs& a, hipStream_t s) {
  long blocks = ((long)a.n + LAUNCH_WAVES - 1) / LAUNCH_WAVES;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) return hipSuccess;
  hipLaunchKernelGGL(launch_kernel, dim3((unsigned)blocks), dim3(LAUNCH_WAVES * 64), 0, s, a);
  return hipGetLastError();
}
#endif  // KP_TU & 1
#if KP_TU & 2
hipError_t launch_feasibility(const FeasArgs& a, hipStream_t s) {
  if (a.bits) {
    if (a.T <= 1024 && !a.one_row) {  // TW <= 16: four rows per wave
      if (a.out_cheapest) {  // seven eval waves and a copy wave for the price rows
        const long blocks = max(((long)a.n_queries + 4 * FEASQ_EW - 1) / (4 * FEASQ_EW), 1L);  // one chunk of rows each
        hipLaunchKernelGGL(feasibility_quad_kernel<FEASQ_EW>, dim3((unsigned)blocks), dim3(FEASB_WAVES * 64), 0, s, a);
      } else {  // no price rows: every wave evaluates
        const long blocks = max(((long)a.n_queries + 4 * FEASB_WAVES - 1) / (4 * FEASB_WAVES), 1L);
        hipLaunchKernelGGL(feasibility_quad_kernel<FEASB_WAVES>, dim3((unsigned)blocks), dim3(FEASB_WAVES * 64), 0, s, a);
      }
    } else {
      hipLaunchKernelGGL(feasibility_bits_kernel, dim3((unsigned)max(1, a.blocks)), dim3(FEASB_WAVES * 64), 0, s, a);
    }
    return hipGetLastError();
  }
  long blocks = ((long)a.n_queries + FEAS_WAVES - 1) / FEAS_WAVES;
  if (blocks > FEAS_MAX_BLOCKS) blocks = FEAS_MAX_BLOCKS;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(feasibility_kernel, dim3((unsigned)blocks), dim3(FEAS_WAVES * 64), 0, s, a);
  return hipGetLastError();
}
#endif  // KP_TU & 2
