// kp_model.h — device data model of the bin-packing hot path (shared by host compile and HIP kernels).
//
// Encoding (DESIGN.md §Data layout):
//  * Label keys get ids 0..K-1 (K <= 64). Keys that ever carry Gt/Lt bounds or minValues get the low ids
//    0..KB-1 (KB <= 16) so their bound slots are dense.
//  * Every (key, value) pair mentioned anywhere in a solve (catalogue requirements, offerings, NodePool
//    requirements/labels, pod selectors/affinities, node labels) gets one bit. Key k owns the
//    WORD-ALIGNED bit range: its first 64 values live in word k, further values in overflow words
//    (ovf[k]..) after the K first words; total words W <= 64, so one wave holds a whole requirement set
//    with one 64-bit word per lane, and "which keys have values" is one __ballot.
//  * An exact scheduling.Requirements value ("kreqs") is: key masks present/complement/has_gt/has_lt/
//    has_min, the bound slots, and the value bitmap vals[W] (upstream Requirement{values, complement,
//    greaterThan, lessThan, MinValues}). Value bits of complement keys hold the NotIn set.
//  * Instance types are a bitmask over the catalogue: TW = ceil(T/64) <= 64 words, one per lane.
//    TM[bit] = the types whose requirement for that key contains that value; DNE[k] = types whose key k
//    is DoesNotExist; NOKEY[k] = types lacking key k.
#pragma once
#include <stdint.h>

#define KP_MAX_KEYS 64
#define KP_MAX_BOUND_KEYS 16
#define KP_MAX_WORDS 64
#define KP_MAX_TYPE_WORDS 64
#define KP_MAX_CLASSES 64
#define KP_SUB_MAX_C 6  // class-subset price table up to 2^6 x T doubles (470 KB at T = 919)
#define KP_NRES 12

struct KReqs {
  uint64_t present, compl_, hgt, hlt, hmin, pad_;
  int64_t gt[KP_MAX_BOUND_KEYS];
  int64_t lt[KP_MAX_BOUND_KEYS];
  int32_t minv[KP_MAX_BOUND_KEYS];
  uint64_t vals[KP_MAX_WORDS];
};

// Offering class = one (capacity-type, zone, zone-id, reservation id, reservation type) signature
// (R:offering.go:133-143, 165-183).
struct OfferClass {  // 16 bytes: two words per class in the LDS catalogue header
  int16_t ct_bit, zone_bit, zid_bit;  // global value bits (< 64 * KP_MAX_WORDS); zid_bit < 0: no zone-id requirement
  int16_t rid_bit, rt_bit;            // capacity-reservation-id / -type value bits; < 0: DoesNotExist
  int16_t pad_[3];
};

// Everything the device needs about the dictionary + one catalogue, for one solve.
struct DevDict {
  int32_t K, W, KB, T, TW, C, R_used, res_any;  // res_any: some offering class is a capacity reservation
  uint64_t wellknown;        // key mask: AllowUndefinedWellKnownLabels
  uint64_t catalog_keys;     // keys some type carries
  uint64_t single_valued;    // catalogue keys where every type has <= 1 value (complement trick allowed)
  uint64_t resid_key_bit;    // 1<<key of karpenter.k8s.aws/capacity-reservation-id (0 if absent)
  uint64_t restype_key_bit;  // 1<<key of ...capacity-reservation-type (0 if absent)
  uint64_t offer_keys;       // keys an offering requirement can name (capacity-type, zone, zone-id, reservation)
  int8_t wkey[KP_MAX_WORDS];     // key of each value word (-1 past W)
  int32_t wofs[KP_MAX_KEYS];     // first word of key k (== k: key k's first value word is word k)
  int32_t ovf[KP_MAX_KEYS];      // first overflow word of key k (keys with > 64 values), -1 if none
  uint64_t firstmask;            // words 0..K-1 (first words)
  uint64_t multiword;            // keys with overflow words
  uint64_t ovfmask[KP_MAX_KEYS]; // overflow words of key k
  int32_t nval[KP_MAX_KEYS];     // values of key k
  uint64_t validbits[KP_MAX_WORDS];  // bits that name a value
  uint64_t vint_ok[KP_MAX_WORDS];    // bits whose value parses with strconv.Atoi
};

// Per-catalogue device arrays (pointers into one device allocation).
struct DevCatalog {
  const uint64_t* TM;       // [nbits(=W*64)][TW]  types containing value bit
  const uint64_t* DNE;      // [K][TW]
  const uint64_t* NOKEY;    // [K][TW]
  const int64_t* vint;      // [W*64] parsed integer of value bit
  const int64_t* alloc;     // [R][T] allocatable milli
  const int64_t* cap;       // [R][T] capacity milli
  const uint64_t* nonneg;   // [TW] types with every allocatable >= 0
  const int64_t* fit_vals;  // [R][T] sorted distinct allocatable values per resource (fit_n[r] used)
  const int32_t* fit_n;     // [R]
  const uint64_t* fit_mask; // [R][T][TW] types with alloc_r >= fit_vals[r][j]
  const OfferClass* cls;    // [C]
  const uint64_t* offer_avail;  // [C][TW] types with an AVAILABLE offering of class c
  const double* price;      // [T][C] price of type t's offering of class c (+inf when none/unavailable)
  const double* price_cm;   // [C][D.T] the same prices class-major (lane = type gathers coalesce)
  const double* price_sub;  // [2^C][D.T] min price over each class subset (C <= KP_SUB_MAX_C), else null
  const uint32_t* name_rank;    // [T] rank of the type name in byte order
  const uint16_t* code;     // [K][T] single-valued code: bit index | 0xFFFE = DNE | 0xFFFF = no key
  const uint64_t* multi;    // [K][T] first-word value mask for multi-valued keys (multi_valued only)
  const uint64_t* custom_nonneg; // [T] key mask of non-well-known keys the type has with a non-NotIn/DNE op
  uint64_t multi_valued;    // keys where some type has > 1 value
  uint64_t custom_any;      // OR of custom_nonneg over the types (0: the per-type test is vacuous)
};
