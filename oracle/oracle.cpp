/*
 * oracle.cpp — CPU restatement of the reference's bin-packing hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline ("kind": "port"). The product (libkp.so) never links
 * or calls it.
 *
 * It is written the way the reference computes: string-keyed maps of string sets (Go
 * map[string]*Requirement with sets.Set[string]), resource maps, per-type scans, Go's pdqsort.
 * Nothing here shares code with the device path's bitset encoding — that is the point.
 *
 * What it restates (file:line in /root/reference, "UP" = sigs.k8s.io/karpenter
 * v1.5.1-0.20250617212656-d0f1c47a99dd pinned at R:go.mod:49, absent from this container; its
 * behaviour is restated from SURVEY.md §8(a) a10-a19 and Appendix B):
 *   - instancetype.NewInstanceType / computeRequirements / computeCapacity / overhead
 *     R:pkg/providers/instancetype/types.go:123-598 (AL2023 family flags R:amifamily/resolver.go:110-117)
 *   - offering.createOfferings R:pkg/providers/instancetype/offering/offering.go:101-150
 *   - filter.CompatibleAvailableFilter / SpotInstanceFilter / ExoticInstanceTypeFilter
 *     R:pkg/providers/instance/filter/filter.go:39-64,279-386
 *   - UP scheduling.Requirement(s): NewRequirementWithFlexibility, Intersection, Len, Operator,
 *     Has, Add, Compatible, Intersects, IsCompatible (call sites R:filter.go:53,59, R:types.go:151)
 *   - UP resources.Fits / Merge / Subtract (call site R:filter.go:56)
 *   - UP Scheduler.Solve / Queue / add / addToExistingNode / addToInflightNode / addToNewNodeClaim /
 *     NodeClaim.Add / ExistingNode.CanAdd / filterInstanceTypesByRequirements / filterByRemainingResources /
 *     subtractMax / Preferences.Relax / Results.TruncateInstanceTypes / InstanceTypes.OrderByPrice /
 *     SatisfiesMinValues  (driver: R:pkg/providers/instancetype/suite_test.go:93,279)
 *   - Go 1.24 sort.Slice (pdqsort_func, zsortfunc.go) — upstream sorts newNodeClaims by len(Pods)
 *     with it before every addToInflightNode.
 *
 * Parity: the catalogue half is pinned by R:website/content/en/preview/reference/instance-types.md
 * (tests/golden/docs_*.tsv) and the KATs of R:pkg/providers/instancetype/suite_test.go; the filter half
 * by R:pkg/providers/instance/filter/filter_test.go (tests/golden/filter_cases.json). Solve tie-breaks
 * (queue order, in-flight order, relaxation order) are "parity unpinned": no Go toolchain and no
 * upstream module here, so this file IS the written spec for them.
 */
#include <arpa/inet.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <regex>
#include <set>
#include <string>
#include <vector>

#include "kp/kp_abi.h"

namespace oracle {

using std::map;
using std::set;
using std::string;
using std::vector;

static const int64_t kMaxInt64 = std::numeric_limits<int64_t>::max();

// ---------------------------------------------------------------------------------------------
// Label keys (R:pkg/apis/v1/labels.go, corev1, karpv1)
// ---------------------------------------------------------------------------------------------
static const char* kLabelZone = "topology.kubernetes.io/zone";
static const char* kLabelRegion = "topology.kubernetes.io/region";
static const char* kLabelInstanceType = "node.kubernetes.io/instance-type";
static const char* kLabelArch = "kubernetes.io/arch";
static const char* kLabelOS = "kubernetes.io/os";
static const char* kLabelWindowsBuild = "node.kubernetes.io/windows-build";
static const char* kLabelCapacityType = "karpenter.sh/capacity-type";
static const char* kLabelNodePool = "karpenter.sh/nodepool";
static const char* kLabelHostname = "kubernetes.io/hostname";  // corev1.LabelHostname
static const char* kLabelZoneID = "topology.k8s.aws/zone-id";
static const char* kLabelResID = "karpenter.k8s.aws/capacity-reservation-id";   // cloudprovider.ReservationIDLabel (R:pkg/apis/v1/doc.go:38)
static const char* kLabelResType = "karpenter.k8s.aws/capacity-reservation-type";
#define AWSL(x) "karpenter.k8s.aws/" x

// karpv1.WellKnownLabels + the AWS insertions of R:pkg/apis/v1/labels.go:31-56.
static const set<string>& WellKnown() {
  static const set<string> s = {
      kLabelNodePool, kLabelZone, kLabelRegion, kLabelInstanceType, kLabelArch, kLabelOS, kLabelCapacityType,
      kLabelWindowsBuild, kLabelResID, kLabelResType, AWSL("instance-hypervisor"),
      AWSL("instance-encryption-in-transit-supported"), AWSL("instance-category"), AWSL("instance-family"),
      AWSL("instance-generation"), AWSL("instance-size"), AWSL("instance-local-nvme"), AWSL("instance-cpu"),
      AWSL("instance-cpu-manufacturer"), AWSL("instance-cpu-sustained-clock-speed-mhz"), AWSL("instance-memory"),
      AWSL("instance-ebs-bandwidth"), AWSL("instance-network-bandwidth"), AWSL("instance-gpu-name"),
      AWSL("instance-gpu-manufacturer"), AWSL("instance-gpu-count"), AWSL("instance-gpu-memory"),
      AWSL("instance-accelerator-name"), AWSL("instance-accelerator-manufacturer"),
      AWSL("instance-accelerator-count"), kLabelZoneID};
  return s;
}

// karpv1.NormalizedLabels (+ the kwok/test-env addition, R:kwok/operator/operator.go:73).
static string Normalize(const string& k) {
  static const map<string, string> m = {
      {"failure-domain.beta.kubernetes.io/zone", kLabelZone},
      {"beta.kubernetes.io/arch", kLabelArch},
      {"beta.kubernetes.io/os", kLabelOS},
      {"beta.kubernetes.io/instance-type", kLabelInstanceType},
      {"failure-domain.beta.kubernetes.io/region", kLabelRegion},
      {"topology.ebs.csi.aws.com/zone", kLabelZone},
  };
  auto it = m.find(k);
  return it == m.end() ? k : it->second;
}

// Go strconv.Atoi (64-bit int): optional sign, decimal digits, no overflow.
static bool GoAtoi(const string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  unsigned __int128 v = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > (unsigned __int128)kMaxInt64 + 1) return false;
  }
  if (!neg && v > (unsigned __int128)kMaxInt64) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// ---------------------------------------------------------------------------------------------
// UP scheduling.Requirement
// ---------------------------------------------------------------------------------------------
struct Requirement {
  string key;
  set<string> values;
  bool complement = false;
  bool has_gt = false, has_lt = false;
  int64_t gt = 0, lt = 0;
  bool has_min = false;
  int min_values = 0;

  int64_t Len() const { return complement ? kMaxInt64 - (int64_t)values.size() : (int64_t)values.size(); }
  // Operator(): Gt/Lt are "Exists with bounds".
  int Op() const {
    if (complement) return Len() < kMaxInt64 ? KP_OP_NOT_IN : KP_OP_EXISTS;
    return Len() > 0 ? KP_OP_IN : KP_OP_DOES_NOT_EXIST;
  }
  bool NegOp() const {
    int o = Op();
    return o == KP_OP_NOT_IN || o == KP_OP_DOES_NOT_EXIST;
  }
};

static bool Within(const string& v, bool hg, int64_t gt, bool hl, int64_t lt) {
  if (!hg && !hl) return true;
  int64_t x;
  if (!GoAtoi(v, &x)) return false;
  if (hg && gt >= x) return false;
  if (hl && lt <= x) return false;
  return true;
}

static bool Has(const Requirement& r, const string& v) {
  bool in = r.values.count(v) > 0;
  if (r.complement) return !in && Within(v, r.has_gt, r.gt, r.has_lt, r.lt);
  return in && Within(v, r.has_gt, r.gt, r.has_lt, r.lt);
}

static Requirement NewRequirement(const string& key_in, int op, const vector<string>& values, int min_values) {
  Requirement r;
  r.key = Normalize(key_in);
  if (min_values >= 0) {
    r.has_min = true;
    r.min_values = min_values;
  }
  if (op == KP_OP_IN) {
    r.values.insert(values.begin(), values.end());
    r.complement = false;
    return r;
  }
  r.complement = !(op == KP_OP_DOES_NOT_EXIST);
  if (op == KP_OP_NOT_IN) r.values.insert(values.begin(), values.end());
  if (op == KP_OP_GT) {
    int64_t x = 0;
    GoAtoi(values.empty() ? "" : values[0], &x);  // prevalidated upstream; Atoi error -> 0
    r.has_gt = true;
    r.gt = x;
  }
  if (op == KP_OP_LT) {
    int64_t x = 0;
    GoAtoi(values.empty() ? "" : values[0], &x);
    r.has_lt = true;
    r.lt = x;
  }
  return r;
}

// Requirement.Intersection.
static Requirement Intersection(const Requirement& a, const Requirement& b) {
  Requirement out;
  out.key = a.key;
  bool comp = a.complement && b.complement;
  bool hg = a.has_gt || b.has_gt, hl = a.has_lt || b.has_lt;
  int64_t gt = 0, lt = 0;
  if (a.has_gt && b.has_gt) gt = std::max(a.gt, b.gt);
  else if (a.has_gt) gt = a.gt;
  else if (b.has_gt) gt = b.gt;
  if (a.has_lt && b.has_lt) lt = std::min(a.lt, b.lt);
  else if (a.has_lt) lt = a.lt;
  else if (b.has_lt) lt = b.lt;
  out.has_min = a.has_min || b.has_min;
  if (a.has_min && b.has_min) out.min_values = std::max(a.min_values, b.min_values);
  else if (a.has_min) out.min_values = a.min_values;
  else if (b.has_min) out.min_values = b.min_values;
  if (hg && hl && gt >= lt) {
    // NewRequirementWithFlexibility(key, DoesNotExist, minValues)
    out.complement = false;
    return out;
  }
  set<string> vals;
  if (a.complement && b.complement) {
    vals = a.values;
    vals.insert(b.values.begin(), b.values.end());
  } else if (a.complement && !b.complement) {
    for (auto& v : b.values)
      if (!a.values.count(v)) vals.insert(v);
  } else if (!a.complement && b.complement) {
    for (auto& v : a.values)
      if (!b.values.count(v)) vals.insert(v);
  } else {
    for (auto& v : a.values)
      if (b.values.count(v)) vals.insert(v);
  }
  for (auto it = vals.begin(); it != vals.end();) {
    if (!Within(*it, hg, gt, hl, lt)) it = vals.erase(it);
    else ++it;
  }
  out.values = std::move(vals);
  out.complement = comp;
  if (comp) {
    out.has_gt = hg;
    out.gt = gt;
    out.has_lt = hl;
    out.lt = lt;
  }
  return out;
}

using Requirements = map<string, Requirement>;

static void Add(Requirements& r, const Requirement& req) {
  auto it = r.find(req.key);
  if (it != r.end()) it->second = Intersection(req, it->second);
  else r[req.key] = req;
}
static void AddAll(Requirements& r, const Requirements& o) {
  for (auto& kv : o) Add(r, kv.second);
}
static bool HasMinValues(const Requirements& r) {
  for (auto& kv : r)
    if (kv.second.has_min) return true;
  return false;
}

// Requirements.Intersects: for every shared key the intersection must be non-empty, unless both
// operators are in {NotIn, DoesNotExist}.
static bool Intersects(const Requirements& r, const Requirements& q) {
  for (auto& kv : r) {
    auto it = q.find(kv.first);
    if (it == q.end()) continue;
    const Requirement& existing = kv.second;
    const Requirement& incoming = it->second;
    if (Intersection(existing, incoming).Len() == 0) {
      if (incoming.NegOp() && existing.NegOp()) continue;
      return false;
    }
  }
  return true;
}

// Requirements.Compatible(q, AllowUndefined?)
static bool Compatible(const Requirements& r, const Requirements& q, bool allow_undefined_wellknown) {
  for (auto& kv : q) {
    if (r.count(kv.first)) continue;
    if (kv.second.NegOp()) continue;
    if (allow_undefined_wellknown && WellKnown().count(kv.first)) continue;
    return false;
  }
  return Intersects(r, q);
}

static Requirements FromABI(const kp_requirements& in) {
  Requirements r;
  for (uint32_t i = 0; i < in.n; i++) {
    const kp_requirement& q = in.items[i];
    vector<string> vals;
    for (uint32_t j = 0; j < q.n_values; j++) vals.push_back(q.values[j] ? q.values[j] : "");
    Add(r, NewRequirement(q.key, q.op, vals, q.min_values));
  }
  return r;
}
static Requirements LabelRequirements(const kp_label* labels, uint32_t n) {
  Requirements r;
  for (uint32_t i = 0; i < n; i++) Add(r, NewRequirement(labels[i].key, KP_OP_IN, {labels[i].value}, -1));
  return r;
}

// ---------------------------------------------------------------------------------------------
// UP resources (map semantics: a missing key is zero)
// ---------------------------------------------------------------------------------------------
using ResourceList = map<int, int64_t>;

static ResourceList FromABI(const kp_resource_list& in) {
  ResourceList r;
  for (int i = 0; i < KP_NUM_RESOURCES; i++)
    if (in.present & (1u << i)) r[i] = in.milli[i];
  return r;
}
static kp_resource_list ToABI(const ResourceList& r) {
  kp_resource_list o;
  memset(&o, 0, sizeof(o));
  for (auto& kv : r) {
    o.milli[kv.first] = kv.second;
    o.present |= 1u << kv.first;
  }
  return o;
}
static int64_t Get(const ResourceList& r, int k) {
  auto it = r.find(k);
  return it == r.end() ? 0 : it->second;
}
static ResourceList Merge(const ResourceList& a, const ResourceList& b) {
  ResourceList o = a;
  for (auto& kv : b) o[kv.first] += kv.second;
  return o;
}
// resources.Subtract(a, b): keys of a, minus b's value when present.
static ResourceList Subtract(const ResourceList& a, const ResourceList& b) {
  ResourceList o = a;
  for (auto& kv : o) kv.second -= Get(b, kv.first);
  return o;
}
// resources.Fits(candidate, total)
static bool Fits(const ResourceList& candidate, const ResourceList& total) {
  for (auto& kv : total)
    if (kv.second < 0) return false;
  for (auto& kv : candidate)
    if (kv.second > Get(total, kv.first)) return false;
  return true;
}

// ---------------------------------------------------------------------------------------------
// Taints (UP scheduling.Taints.ToleratesPod + corev1 Toleration.ToleratesTaint)
// ---------------------------------------------------------------------------------------------
struct Taint {
  string key, value;
  int effect;
};
struct Toleration {
  string key, value;
  int op, effect;
};
static bool ToleratesTaint(const Toleration& t, const Taint& taint) {
  if (t.effect != KP_EFFECT_ANY && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op == KP_TOL_EQUAL) return t.value == taint.value;
  if (t.op == KP_TOL_EXISTS) return true;
  return false;
}
static bool ToleratesAll(const vector<Taint>& taints, const vector<Toleration>& tols) {
  for (auto& taint : taints) {
    bool ok = false;
    for (auto& t : tols) ok = ok || ToleratesTaint(t, taint);
    if (!ok) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// cloudprovider.InstanceType / Offering (UP pkg/cloudprovider/types.go)
// ---------------------------------------------------------------------------------------------
struct Offering {
  Requirements reqs;
  double price;
  bool available;
  int32_t reservation_capacity = 0;  // Offering.ReservationCapacity (R:offering.go:178)
};
struct InstanceType {
  string name;
  Requirements reqs;
  ResourceList capacity, overhead, allocatable;
  vector<Offering> offerings;
};

static std::shared_ptr<vector<InstanceType>> CatalogFromABI(const kp_catalog_desc& d) {
  auto out = std::make_shared<vector<InstanceType>>();
  out->reserve(d.n_types);
  for (uint32_t i = 0; i < d.n_types; i++) {
    const kp_instance_type& t = d.types[i];
    InstanceType it;
    it.name = t.name;
    it.reqs = FromABI(t.requirements);
    it.capacity = FromABI(t.capacity);
    it.overhead = FromABI(t.overhead);
    it.allocatable = Subtract(it.capacity, it.overhead);  // InstanceType.Allocatable()
    for (uint32_t j = 0; j < t.n_offerings; j++) {
      const kp_offering& o = t.offerings[j];
      Offering of;
      Add(of.reqs, NewRequirement(kLabelCapacityType, KP_OP_IN, {o.capacity_type}, -1));
      if (o.zone) Add(of.reqs, NewRequirement(kLabelZone, KP_OP_IN, {o.zone}, -1));
      if (o.reservation_id) Add(of.reqs, NewRequirement(kLabelResID, KP_OP_IN, {o.reservation_id}, -1));
      else Add(of.reqs, NewRequirement(kLabelResID, KP_OP_DOES_NOT_EXIST, {}, -1));
      if (o.reservation_type) Add(of.reqs, NewRequirement(kLabelResType, KP_OP_IN, {o.reservation_type}, -1));
      else Add(of.reqs, NewRequirement(kLabelResType, KP_OP_DOES_NOT_EXIST, {}, -1));
      if (o.zone_id) Add(of.reqs, NewRequirement(kLabelZoneID, KP_OP_IN, {o.zone_id}, -1));
      of.price = o.price;
      of.available = o.available != 0;
      of.reservation_capacity = o.reservation_capacity;
      it.offerings.push_back(std::move(of));
    }
    out->push_back(std::move(it));
  }
  return out;
}

// Offerings.Available().Compatible(reqs) non-empty (R:filter.go:59; UP filterInstanceTypesByRequirements)
static bool HasCompatibleAvailable(const InstanceType& it, const Requirements& reqs) {
  for (auto& o : it.offerings)
    if (o.available && Compatible(reqs, o.reqs, true)) return true;
  return false;
}
// Cheapest compatible available offering price, MaxFloat64 when none (UP OrderByPrice).
static double CheapestPrice(const InstanceType& it, const Requirements& reqs) {
  double p = std::numeric_limits<double>::max();
  bool any = false;
  for (auto& o : it.offerings)
    if (o.available && Compatible(reqs, o.reqs, true)) {
      if (!any || o.price < p) p = o.price;
      any = true;
    }
  return p;
}

// ---------------------------------------------------------------------------------------------
// Go sort.Slice — pdqsort_func (Go 1.24 src/sort/zsortfunc.go), restated over less/swap.
// ---------------------------------------------------------------------------------------------
template <class LS>
struct PDQ {
  LS& d;
  enum { increasingHint, decreasingHint, unknownHint };
  void insertionSort(int a, int b) {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && d.Less(j, j - 1); j--) d.Swap(j, j - 1);
  }
  void siftDown(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && d.Less(first + child, first + child + 1)) child++;
      if (!d.Less(first + root, first + child)) return;
      d.Swap(first + root, first + child);
      root = child;
    }
  }
  void heapSort(int a, int b) {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      d.Swap(first, first + i);
      siftDown(lo, i, first);
    }
  }
  static int bitsLen(uint64_t x) { return x == 0 ? 0 : 64 - __builtin_clzll(x); }
  void breakPatterns(int a, int b) {
    int length = b - a;
    if (length >= 8) {
      uint64_t random = (uint64_t)length;
      uint64_t modulus = 1ull << bitsLen((uint64_t)length);
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        random ^= random << 13;
        random ^= random >> 7;
        random ^= random << 17;
        int other = (int)((unsigned)random & (unsigned)(modulus - 1));
        if (other >= length) other -= length;
        d.Swap(idx - 1 + i, a + other);
      }
    }
  }
  void order2(int& a, int& b, int* swaps) {
    if (d.Less(b, a)) {
      (*swaps)++;
      std::swap(a, b);
    }
  }
  int median(int a, int b, int c, int* swaps) {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  int medianAdjacent(int a, int* swaps) { return median(a - 1, a, a + 1, swaps); }
  int choosePivot(int a, int b, int* hint) {
    const int shortestNinther = 50, maxSwaps = 4 * 3;
    int l = b - a, swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= shortestNinther) {
        i = medianAdjacent(i, &swaps);
        j = medianAdjacent(j, &swaps);
        k = medianAdjacent(k, &swaps);
      }
      j = median(i, j, k, &swaps);
    }
    *hint = swaps == 0 ? increasingHint : (swaps == maxSwaps ? decreasingHint : unknownHint);
    return j;
  }
  void reverseRange(int a, int b) {
    int i = a, j = b - 1;
    while (i < j) d.Swap(i++, j--);
  }
  bool partialInsertionSort(int a, int b) {
    const int maxSteps = 5, shortestShifting = 50;
    int i = a + 1;
    for (int j = 0; j < maxSteps; j++) {
      while (i < b && !d.Less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < shortestShifting) return false;
      d.Swap(i, i - 1);
      if (i - a >= 2) {
        for (int k = i - 1; k >= 1; k--) {
          if (!d.Less(k, k - 1)) break;
          d.Swap(k, k - 1);
        }
      }
      if (b - i >= 2) {
        for (int k = i + 1; k < b; k++) {
          if (!d.Less(k, k - 1)) break;
          d.Swap(k, k - 1);
        }
      }
    }
    return false;
  }
  int partitionEqual(int a, int b, int pivot) {
    d.Swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !d.Less(a, i)) i++;
      while (i <= j && d.Less(a, j)) j--;
      if (i > j) break;
      d.Swap(i, j);
      i++;
      j--;
    }
    return i;
  }
  int partition(int a, int b, int pivot, bool* already) {
    d.Swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.Less(i, a)) i++;
    while (i <= j && !d.Less(j, a)) j--;
    if (i > j) {
      d.Swap(j, a);
      *already = true;
      return j;
    }
    d.Swap(i, j);
    i++;
    j--;
    for (;;) {
      while (i <= j && d.Less(i, a)) i++;
      while (i <= j && !d.Less(j, a)) j--;
      if (i > j) break;
      d.Swap(i, j);
      i++;
      j--;
    }
    d.Swap(j, a);
    *already = false;
    return j;
  }
  void pdqsort(int a, int b, int limit) {
    const int maxInsertion = 12;
    bool wasBalanced = true, wasPartitioned = true;
    for (;;) {
      int length = b - a;
      if (length <= maxInsertion) {
        insertionSort(a, b);
        return;
      }
      if (limit == 0) {
        heapSort(a, b);
        return;
      }
      if (!wasBalanced) {
        breakPatterns(a, b);
        limit--;
      }
      int hint;
      int pivot = choosePivot(a, b, &hint);
      if (hint == decreasingHint) {
        reverseRange(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = increasingHint;
      }
      if (wasBalanced && wasPartitioned && hint == increasingHint) {
        if (partialInsertionSort(a, b)) return;
      }
      if (a > 0 && !d.Less(a - 1, pivot)) {
        int mid = partitionEqual(a, b, pivot);
        a = mid;
        continue;
      }
      bool already = false;
      int mid = partition(a, b, pivot, &already);
      wasPartitioned = already;
      int leftLen = mid - a, rightLen = b - mid;
      int balanceThreshold = length / 8;
      if (leftLen < rightLen) {
        wasBalanced = leftLen >= balanceThreshold;
        pdqsort(a, mid, limit);
        a = mid + 1;
      } else {
        wasBalanced = rightLen >= balanceThreshold;
        pdqsort(mid + 1, b, limit);
        b = mid;
      }
    }
  }
};
template <class LS>
static void GoSortSlice(LS& ls, int n) {
  PDQ<LS> p{ls};
  p.pdqsort(0, n, PDQ<LS>::bitsLen((uint64_t)n));
}

// ---------------------------------------------------------------------------------------------
// UP scheduler
// ---------------------------------------------------------------------------------------------
struct Template {
  int nodepool;       // index into input nodepools
  string name;
  int weight;
  Requirements reqs;  // NewNodeClaimTemplate
  vector<Taint> taints;
  const vector<InstanceType>* catalog;
  vector<int> options;  // InstanceTypeOptions (indices into catalog)
  ResourceList daemon;
  bool has_limits;
  ResourceList remaining;
};

// ---------------------------------------------------------------------------------------------
// metav1.LabelSelector (labels.Selector from LabelSelectorAsSelector)
// ---------------------------------------------------------------------------------------------
struct SelReq {
  string key;
  int op;
  set<string> values;
};
struct Selector {
  bool nil = true;
  vector<SelReq> reqs;  // matchLabels become In{v}
  bool Matches(const map<string, string>& labels) const {
    if (nil) return false;  // labels.Nothing()
    for (auto& r : reqs) {
      auto it = labels.find(r.key);
      const bool has = it != labels.end();
      switch (r.op) {
        case KP_SEL_IN:
          if (!has || !r.values.count(it->second)) return false;
          break;
        case KP_SEL_NOT_IN:
          if (has && r.values.count(it->second)) return false;
          break;
        case KP_SEL_EXISTS:
          if (!has) return false;
          break;
        default:
          if (has) return false;
      }
    }
    return true;
  }
  string Canon() const {
    if (nil) return "nil";
    vector<string> parts;
    for (auto& r : reqs) {
      string x = r.key + "/" + std::to_string(r.op);
      for (auto& v : r.values) x += "," + v;
      parts.push_back(x);
    }
    std::sort(parts.begin(), parts.end());
    string o;
    for (auto& x : parts) o += x + ";";
    return o;
  }
};

struct Spread {
  string key;
  int32_t maxSkew, minDomains;  // minDomains < 0: nil
  int when, affinityPolicy, taintsPolicy;
  Selector sel;
};
// corev1.PodAffinityTerm of a podAntiAffinity (TopologyTypePodAntiAffinity)
struct AntiTerm {
  string key;
  Selector sel;
  set<string> namespaces;  // buildNamespaceList: the term's namespaces, else the pod's own
  int32_t weight;
};
static Selector SelectorFromABI(const kp_label_selector& s) {
  Selector o;
  o.nil = s.is_nil != 0;
  for (uint32_t k = 0; k < s.n_match_labels; k++)
    o.reqs.push_back({s.match_labels[k].key, KP_SEL_IN, {s.match_labels[k].value ? s.match_labels[k].value : ""}});
  for (uint32_t k = 0; k < s.n_match_expressions; k++) {
    const kp_selector_requirement& e = s.match_expressions[k];
    SelReq r{e.key, e.op, {}};
    for (uint32_t v = 0; v < e.n_values; v++) r.values.insert(e.values[v] ? e.values[v] : "");
    o.reqs.push_back(r);
  }
  return o;
}
// The cluster's namespaces (kp_solve_in.namespaces) a namespaceSelector lists.
struct NamespaceList {
  vector<std::pair<string, map<string, string>>> items;
};
static NamespaceList NamespacesFromABI(const kp_namespace* ns, uint32_t n) {
  NamespaceList o;
  for (uint32_t i = 0; i < n; i++) {
    map<string, string> l;
    for (uint32_t j = 0; j < ns[i].n_labels; j++) l[ns[i].labels[j].key] = ns[i].labels[j].value ? ns[i].labels[j].value : "";
    o.items.push_back({ns[i].name ? ns[i].name : "", l});
  }
  return o;
}
// UP Topology.buildNamespaceList: no namespaces and no namespaceSelector -> the pod's own namespace; otherwise the
// term's namespaces plus every namespace the namespaceSelector selects (kubeClient.List with its LabelSelector)
static AntiTerm AntiFromABI(const kp_pod_affinity_term& t, const string& podNs, const NamespaceList& nsl) {
  AntiTerm a;
  a.key = t.topology_key ? t.topology_key : "";
  a.sel = SelectorFromABI(t.selector);
  for (uint32_t i = 0; i < t.n_namespaces; i++) a.namespaces.insert(t.namespaces[i] ? t.namespaces[i] : "");
  if (t.has_namespace_selector) {
    const Selector ns = SelectorFromABI(t.namespace_selector);
    for (auto& item : nsl.items)
      if (ns.Matches(item.second)) a.namespaces.insert(item.first);
  } else if (a.namespaces.empty()) {
    a.namespaces.insert(podNs);
  }
  a.weight = t.weight;
  return a;
}

// UP scheduling.HostPort / GetHostPorts / HostPortUsage (hostportusage.go): hostIP "" -> 0.0.0.0, protocol "" -> TCP,
// hostPort 0 skipped; Matches = same protocol and port, and an unspecified IP on either side or equal IPs
// (net.IP.Equal: an IPv4 address equals its v4-in-v6 form).
struct HostPort {
  int proto, port;
  unsigned char ip[16];  // net.ParseIP form: IPv4 as ::ffff:a.b.c.d
  bool IsUnspecified() const {
    static const unsigned char z[16] = {0};
    static const unsigned char z4[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF, 0, 0, 0, 0};
    return !memcmp(ip, z, 16) || !memcmp(ip, z4, 16);
  }
  bool Matches(const HostPort& r) const {
    if (proto != r.proto || port != r.port) return false;
    if (IsUnspecified() || r.IsUnspecified()) return true;
    return !memcmp(ip, r.ip, 16);
  }
};
static bool GetHostPorts(const kp_host_port* hp, uint32_t n, vector<HostPort>* out) {
  for (uint32_t i = 0; i < n; i++) {
    if (hp[i].port == 0) continue;
    HostPort h;
    h.proto = hp[i].protocol;
    h.port = hp[i].port;
    memset(h.ip, 0, 16);
    const char* ip = hp[i].ip && hp[i].ip[0] ? hp[i].ip : "0.0.0.0";
    unsigned char v4[4];
    if (inet_pton(AF_INET, ip, v4) == 1) {
      h.ip[10] = h.ip[11] = 0xFF;
      memcpy(h.ip + 12, v4, 4);
    } else if (inet_pton(AF_INET6, ip, h.ip) != 1) {
      return false;
    }
    out->push_back(h);
  }
  return true;
}
// HostPortUsage.Conflicts(pod, ports): any new entry matching an entry another pod reserved
static bool HostPortsConflict(const vector<HostPort>& reserved, const vector<HostPort>& ports) {
  for (auto& n : ports)
    for (auto& e : reserved)
      if (n.Matches(e)) return true;
  return false;
}

struct PodState {
  int index;
  int shape;
  int64_t cpu, mem;  // sort keys
  int64_t creation;
  uint64_t uid;
  string uid_str;  // metadata.uid when the batch passes it (kp_solve_in.pod_uids): compared as a string
  // relaxable spec (Preferences.Relax mutates the pod)
  vector<Requirements> required_terms;
  vector<std::pair<int, Requirements>> preferred;  // (weight, preference)
  Requirements node_selector;
  ResourceList requests;
  vector<Toleration> tolerations;
  vector<Spread> spreads;
  vector<AntiTerm> antiRequired, antiPreferred;  // podAntiAffinity (preferred: relaxed heaviest first)
  vector<AntiTerm> affRequired, affPreferred;    // podAffinity (same term shape)
  string ns;
  map<string, string> labels;
  vector<HostPort> hostPorts;
  Requirements reqs;    // cached NewPodRequirements
  Requirements strict;  // cached NewStrictPodRequirements (no preferred terms)
};

// NewPodRequirements (UP scheduling/requirements.go): nodeSelector + heaviest preferred term (treated
// as required) + the first required term. Strict: without the preferred term.
static Requirements PodRequirements(PodState& p) {
  Requirements r = p.node_selector;
  if (!p.preferred.empty()) {
    // sort.Slice(preferred, weight desc) mutates the pod; len <= 12 is insertion sort (stable)
    struct LS {
      vector<std::pair<int, Requirements>>& v;
      bool Less(int i, int j) { return v[i].first > v[j].first; }
      void Swap(int i, int j) { std::swap(v[i], v[j]); }
    } ls{p.preferred};
    GoSortSlice(ls, (int)p.preferred.size());
    AddAll(r, p.preferred[0].second);
  }
  if (!p.required_terms.empty()) AddAll(r, p.required_terms[0]);
  return r;
}
static Requirements StrictPodRequirements(const PodState& p) {
  Requirements r = p.node_selector;
  if (!p.required_terms.empty()) AddAll(r, p.required_terms[0]);
  return r;
}

// Preferences.Relax (UP preferences.go): first applicable of removeRequiredNodeAffinityTerm (only when
// >1 terms), removePreferredPodAffinityTerm, removePreferredPodAntiAffinityTerm (heaviest first),
// removePreferredNodeAffinityTerm (heaviest), removeTopologySpreadScheduleAnyway (first ScheduleAnyway
// constraint, swap-with-last removal), and, only when Preferences.ToleratePreferNoSchedule is set (NewScheduler:
// some NodePool template taint has effect PreferNoSchedule), toleratePreferNoScheduleTaints.
// Order of the preferred terms: the docs say "by ascending weight (lowest weight is relaxed first)"
// (R:website/content/en/preview/concepts/scheduling.md:216); the upstream code sorts them by weight descending
// and removes element 0, the heaviest. The code is followed: NewPodRequirements applies only the heaviest
// preferred term as a requirement, so dropping the lightest one first would leave the failing requirement in
// place and change nothing (DESIGN.md §2 records the conflict).
static bool Relax(PodState& p, bool toleratePNS) {
  if (p.required_terms.size() > 1) {
    p.required_terms.erase(p.required_terms.begin());
    return true;
  }
  if (!p.affPreferred.empty()) {  // removePreferredPodAffinityTerm: sort.Slice by weight desc (<= 12: stable)
    std::stable_sort(p.affPreferred.begin(), p.affPreferred.end(),
                     [](const AntiTerm& a, const AntiTerm& b) { return a.weight > b.weight; });
    p.affPreferred.erase(p.affPreferred.begin());
    return true;
  }
  if (!p.antiPreferred.empty()) {  // removePreferredPodAntiAffinityTerm: sort.Slice by weight desc (<= 12: stable)
    std::stable_sort(p.antiPreferred.begin(), p.antiPreferred.end(),
                     [](const AntiTerm& a, const AntiTerm& b) { return a.weight > b.weight; });
    p.antiPreferred.erase(p.antiPreferred.begin());
    return true;
  }
  if (!p.preferred.empty()) {
    std::stable_sort(p.preferred.begin(), p.preferred.end(),
                     [](const std::pair<int, Requirements>& a, const std::pair<int, Requirements>& b) {
                       return a.first > b.first;
                     });
    p.preferred.erase(p.preferred.begin());
    return true;
  }
  for (size_t i = 0; i < p.spreads.size(); i++)
    if (p.spreads[i].when == KP_SCHEDULE_ANYWAY) {
      p.spreads[i] = p.spreads.back();
      p.spreads.pop_back();
      return true;
    }
  if (toleratePNS) {  // toleratePreferNoScheduleTaints: {Operator: Exists, Effect: PreferNoSchedule}
    for (auto& t : p.tolerations)  // corev1 Toleration.MatchToleration: key, operator, value, effect all equal
      if (t.key.empty() && t.value.empty() && t.op == KP_TOL_EXISTS && t.effect == KP_EFFECT_PREFER_NO_SCHEDULE)
        return false;
    p.tolerations.push_back({"", "", KP_TOL_EXISTS, KP_EFFECT_PREFER_NO_SCHEDULE});
    return true;
  }
  return false;
}

static Requirement ExistsReq(const string& key) { return NewRequirement(key, KP_OP_EXISTS, {}, -1); }
static const Requirement& GetOr(const Requirements& r, const string& key, Requirement& tmp) {
  auto it = r.find(key);
  if (it != r.end()) return it->second;
  tmp = ExistsReq(key);
  return tmp;
}

// ---------------------------------------------------------------------------------------------
// UP Topology / TopologyGroup (topology.go, topologygroup.go, topologynodefilter.go,
// topologydomaingroup.go) for TopologyTypeSpread. Tie-break: where upstream iterates a Go map or an
// unsorted set (equal counts), the lexicographically smallest domain is chosen.
// ---------------------------------------------------------------------------------------------
struct TopologyGroup {
  string key, id;
  int type = 0;  // 0 TopologyTypeSpread, 1 TopologyTypePodAffinity, 2 TopologyTypePodAntiAffinity
  set<string> nss;  // anti-affinity: the term's namespaces
  int32_t maxSkew, minDomains;
  string ns;
  Selector sel;
  vector<Requirements> filter;  // TopologyNodeFilter.Requirements (ORed)
  bool affinityHonor, taintHonor;
  vector<Toleration> tols;
  map<string, int32_t> domains;
  set<int> owners;

  bool Selects(const string& pns, const map<string, string>& labels) const {
    return (type != 0 ? nss.count(pns) > 0 : pns == ns) && sel.Matches(labels);
  }
  bool FilterMatches(const vector<Taint>& taints, const Requirements& reqs, bool allow) const {
    bool aff = true;
    if (affinityHonor && !filter.empty()) {
      aff = false;
      for (auto& f : filter)
        if (Compatible(reqs, f, allow)) {
          aff = true;
          break;
        }
    }
    const bool tnt = !taintHonor || ToleratesAll(taints, tols);
    return aff && tnt;
  }
  int64_t DomainMinCount(const Requirement& podDomains) const {
    if (key == kLabelHostname) return 0;  // hostname topologies can always create a new domain
    int64_t mn = std::numeric_limits<int32_t>::max();
    int32_t num = 0;
    for (auto& kv : domains)
      if (Has(podDomains, kv.first)) {
        num++;
        mn = std::min<int64_t>(mn, kv.second);
      }
    if (minDomains >= 0 && num < minDomains) mn = 0;
    return mn;
  }
  // nextDomainAntiAffinity: every known domain the pod admits whose count is zero
  Requirement NextDomainAnti(const Requirement& podDomains) const {
    vector<string> options;
    for (auto& kv : domains)
      if (Has(podDomains, kv.first) && kv.second == 0) options.push_back(kv.first);
    if (options.empty()) return NewRequirement(key, KP_OP_DOES_NOT_EXIST, {}, -1);
    return NewRequirement(key, KP_OP_IN, options, -1);
  }
  // nextDomainAffinity: the known domains the pod admits that hold a selected pod; none and the pod selects itself:
  // bootstrap with the first domain of podDomains ∩ nodeDomains and the first of podDomains (upstream iterates a
  // map there: the lexicographically smallest, as everywhere in this oracle)
  Requirement NextDomainAffinity(bool self, const Requirement& podDomains, const Requirement& nodeDomains) const {
    vector<string> options;
    for (auto& kv : domains)
      if (Has(podDomains, kv.first) && kv.second > 0) options.push_back(kv.first);
    if (options.empty() && self) {
      for (auto& kv : domains)
        if (Has(podDomains, kv.first) && Has(nodeDomains, kv.first)) {
          options.push_back(kv.first);
          break;
        }
      for (auto& kv : domains)
        if (Has(podDomains, kv.first)) {
          if (std::find(options.begin(), options.end(), kv.first) == options.end()) options.push_back(kv.first);
          break;
        }
    }
    if (options.empty()) return NewRequirement(key, KP_OP_DOES_NOT_EXIST, {}, -1);
    return NewRequirement(key, KP_OP_IN, options, -1);
  }
  // nextDomainTopologySpread
  Requirement NextDomain(bool self, const Requirement& podDomains, const Requirement& nodeDomains) const {
    if (type == 2) return NextDomainAnti(podDomains);
    if (type == 1) return NextDomainAffinity(self, podDomains, nodeDomains);
    const int64_t mn = DomainMinCount(podDomains);
    string minDomain;
    bool found = false;
    int64_t minCount = std::numeric_limits<int32_t>::max();
    auto consider = [&](const string& d, int32_t c) {
      const int64_t count = (int64_t)c + (self ? 1 : 0);
      if (count - mn <= maxSkew && count < minCount) {
        minDomain = d;
        minCount = count;
        found = true;
      }
    };
    if (nodeDomains.Op() == KP_OP_IN) {
      for (auto& v : nodeDomains.values) {  // sorted
        auto it = domains.find(v);
        if (it != domains.end()) consider(v, it->second);
      }
    } else {
      for (auto& kv : domains)
        if (Has(nodeDomains, kv.first)) consider(kv.first, kv.second);
    }
    if (!found) return NewRequirement(key, KP_OP_DOES_NOT_EXIST, {}, -1);
    return NewRequirement(key, KP_OP_IN, {minDomain}, -1);
  }
};

struct BoundPod {
  string ns;
  map<string, string> labels;
  int node;  // input index of the existing node
  vector<AntiTerm> anti;  // its required podAntiAffinity terms (inverse groups)
};
struct NodeView {  // what countDomains reads of a node
  string name;
  map<string, string> labels;
  vector<Taint> taints;
  Requirements reqs;  // NewLabelRequirements(labels)
};

struct Topology {
  vector<std::unique_ptr<TopologyGroup>> groups;  // creation order
  map<string, TopologyGroup*> byId;
  map<string, map<string, vector<vector<Taint>>>> domainGroups;  // key -> domain -> taint sets
  vector<BoundPod> bound;
  vector<NodeView> nodes;

  static string ReqsCanon(const Requirements& r) {
    string o;
    for (auto& kv : r) {
      const Requirement& q = kv.second;
      o += kv.first + (q.complement ? "!" : "=");
      for (auto& v : q.values) o += v + ",";
      if (q.has_gt) o += ">" + std::to_string(q.gt);
      if (q.has_lt) o += "<" + std::to_string(q.lt);
      if (q.has_min) o += "#" + std::to_string(q.min_values);
      o += ";";
    }
    return o;
  }

  // MakeTopologyNodeFilter + NewTopologyGroup; identity = upstream TopologyGroup.Hash fields (key, type,
  // namespaces, selector, maxSkew, node filter = requirements, both policies and the pod's tolerations).
  std::unique_ptr<TopologyGroup> NewGroup(const PodState& p, const Spread& s) const {
    auto g = std::make_unique<TopologyGroup>();
    g->key = s.key;
    g->maxSkew = s.maxSkew;
    g->minDomains = s.minDomains;
    g->ns = p.ns;
    g->sel = s.sel;
    g->affinityHonor = s.affinityPolicy != KP_POLICY_IGNORE;
    g->taintHonor = s.taintsPolicy == KP_POLICY_HONOR;
    g->tols = p.tolerations;
    if (p.required_terms.empty()) {
      g->filter.push_back(p.node_selector);
    } else {
      for (auto& t : p.required_terms) {
        Requirements r = p.node_selector;
        AddAll(r, t);
        g->filter.push_back(r);
      }
    }
    string id = s.key + "|" + std::to_string(s.maxSkew) + "|" + p.ns + "|" + s.sel.Canon() + "|" +
                std::to_string(g->affinityHonor) + std::to_string(g->taintHonor) + "|";
    for (auto& f : g->filter) id += "[" + ReqsCanon(f) + "]";
    // the filter's tolerations under every taint policy (upstream TopologyNodeFilter.Tolerations, hashed with it)
    for (auto& t : g->tols) id += "(" + t.key + "," + t.value + "," + std::to_string(t.op) + "," + std::to_string(t.effect) + ")";
    g->id = id;
    // domainGroup.ForEachDomain(pod, taintPolicy): register every known domain with a zero count
    auto dg = domainGroups.find(s.key);
    if (dg != domainGroups.end())
      for (auto& kv : dg->second) {
        bool ok = !g->taintHonor;
        for (size_t i = 0; i < kv.second.size() && !ok; i++) ok = ToleratesAll(kv.second[i], p.tolerations);
        if (ok) g->domains.emplace(kv.first, 0);
      }
    return g;
  }

  // NewTopologyGroup(TopologyTypePodAntiAffinity, ...): no node filter, every known domain registered; identity =
  // (type, key, namespaces, selector)
  std::unique_ptr<TopologyGroup> NewAntiGroup(const AntiTerm& t, int type = 2) const {
    auto g = std::make_unique<TopologyGroup>();
    g->type = type;
    g->key = t.key;
    g->maxSkew = std::numeric_limits<int32_t>::max();
    g->minDomains = -1;
    g->sel = t.sel;
    g->nss = t.namespaces;
    g->affinityHonor = false;
    g->taintHonor = false;
    string id = (type == 1 ? "aff|" : "anti|") + t.key + "|";
    for (auto& n : t.namespaces) id += n + ",";
    g->id = id + "|" + t.sel.Canon();
    auto dg = domainGroups.find(t.key);
    if (dg != domainGroups.end())
      for (auto& kv : dg->second) g->domains.emplace(kv.first, 0);
    return g;
  }
  vector<std::unique_ptr<TopologyGroup>> inverse;  // updateInverseAntiAffinity: bound pods' required terms
  map<string, TopologyGroup*> inverseById;
  void BuildInverse() {
    for (auto& bp : bound)
      for (auto& t : bp.anti) {
        auto g = NewAntiGroup(t);
        TopologyGroup* tg;
        auto it = inverseById.find(g->id);
        if (it == inverseById.end()) {
          tg = g.get();
          inverseById[g->id] = tg;
          inverse.push_back(std::move(g));
        } else {
          tg = it->second;
        }
        const NodeView& n = nodes[(size_t)bp.node];
        auto lv = n.labels.find(t.key);
        if (lv != n.labels.end()) tg->domains[lv->second]++;
        else if (t.key == kLabelHostname) tg->domains[n.name]++;
      }
  }

  // countDomains: pods already running that the group selects, on nodes the filter admits; then every
  // existing node's domain value with a zero count.
  void CountDomains(TopologyGroup& g) const {
    for (auto& bp : bound) {
      if (!g.Selects(bp.ns, bp.labels)) continue;
      const NodeView& n = nodes[(size_t)bp.node];
      auto it = n.labels.find(g.key);
      string domain;
      if (it != n.labels.end()) domain = it->second;
      else if (g.key == kLabelHostname) domain = n.name;
      else continue;
      if (!g.FilterMatches(n.taints, n.reqs, false)) continue;
      g.domains[domain]++;
    }
    for (auto& n : nodes) {
      if (!g.FilterMatches(n.taints, n.reqs, false)) continue;
      auto it = n.labels.find(g.key);
      if (it == n.labels.end()) continue;
      g.domains.emplace(it->second, 0);
    }
  }

  // Topology.Update: the pod stops owning every group, then owns the groups of its current spreads
  void Update(const PodState& p) {
    for (auto& g : groups) g->owners.erase(p.index);
    vector<std::unique_ptr<TopologyGroup>> fresh;
    for (auto& s : p.spreads) fresh.push_back(NewGroup(p, s));
    for (auto& t : p.antiRequired) fresh.push_back(NewAntiGroup(t));
    for (auto& t : p.antiPreferred) fresh.push_back(NewAntiGroup(t));
    for (auto& t : p.affRequired) fresh.push_back(NewAntiGroup(t, 1));
    for (auto& t : p.affPreferred) fresh.push_back(NewAntiGroup(t, 1));
    for (auto& g : fresh) {
      auto it = byId.find(g->id);
      TopologyGroup* tg;
      if (it == byId.end()) {
        CountDomains(*g);
        tg = g.get();
        byId[g->id] = tg;
        groups.push_back(std::move(g));
      } else {
        tg = it->second;
      }
      tg->owners.insert(p.index);
    }
  }
  void Register(const string& key, const string& domain) {  // topologies and inverseTopologies alike
    for (auto& g : groups)
      if (g->key == key) g->domains.emplace(domain, 0);
    for (auto& g : inverse)
      if (g->key == key) g->domains.emplace(domain, 0);
  }
  void Unregister(const string& key, const string& domain) {
    for (auto& g : groups)
      if (g->key == key) g->domains.erase(domain);
    for (auto& g : inverse)
      if (g->key == key) g->domains.erase(domain);
  }
  // AddRequirements: every group the pod owns narrows its key to the chosen domain
  bool AddRequirements(const PodState& p, const Requirements& nodeReqs, Requirements* out) const {
    *out = nodeReqs;
    vector<const TopologyGroup*> matching;  // getMatchingTopologies: owned groups, then inverse groups selecting p
    for (auto& g : groups)
      if (g->owners.count(p.index)) matching.push_back(g.get());
    for (auto& g : inverse)
      if (g->Selects(p.ns, p.labels)) matching.push_back(g.get());
    for (const TopologyGroup* g : matching) {
      Requirement t1, t2;
      const Requirement& podDomains = GetOr(p.strict, g->key, t1);
      const Requirement& nodeDomains = GetOr(nodeReqs, g->key, t2);
      Requirement d = g->NextDomain(g->Selects(p.ns, p.labels), podDomains, nodeDomains);
      if (d.Len() == 0) return false;
      Add(*out, d);
    }
    return true;
  }
  // Record: every group that counts the pod on a node with these requirements (single-domain keys only)
  void Record(const PodState& p, const vector<Taint>& taints, const Requirements& reqs, bool allow) {
    for (auto& g : groups) {
      if (!g->Selects(p.ns, p.labels) || !g->FilterMatches(taints, reqs, allow)) continue;
      auto it = reqs.find(g->key);
      if (g->type == 2) {  // anti-affinity blocks every domain the node could be in: Record(domains.Values()...)
        if (it != reqs.end())
          for (auto& v : it->second.values) g->domains[v]++;
        continue;
      }
      if (it == reqs.end() || it->second.Len() != 1) continue;
      g->domains[*it->second.values.begin()]++;
    }
  }
};

struct NodeClaim {
  int id;  // creation order
  const Template* tmpl;
  Requirements reqs;
  vector<int> options;
  ResourceList requests;
  vector<int> pods;
  string hostname;
  vector<HostPort> hostPortUsage;
  set<string> reserved;  // NodeClaim.reservedOfferings, by reservation id (an id names one offering of one type)
  // max allocatable per resource over `options` (missing = 0): a checker-side shortcut, not part of the restated
  // algorithm. If the merged requests exceed it on some resource, no option Fits, so filterInstanceTypesByRequirements
  // returns nothing and NodeClaim.Add fails whatever the requirement checks say; the outcome is unchanged.
  int64_t maxalloc[KP_NUM_RESOURCES] = {};
};

static void SetMaxAlloc(NodeClaim& n) {
  for (int r = 0; r < KP_NUM_RESOURCES; r++) n.maxalloc[r] = INT64_MIN;
  for (int t : n.options)
    for (int r = 0; r < KP_NUM_RESOURCES; r++) n.maxalloc[r] = std::max(n.maxalloc[r], Get((*n.tmpl->catalog)[t].allocatable, r));
}

struct ExistingNode {
  int index;  // input index
  string name;
  bool initialized;
  Requirements reqs;
  vector<Taint> taints;
  ResourceList available, requests;
  vector<int> pods;
  vector<HostPort> hostPortUsage;
};

static bool SatisfiesMinValues(const vector<InstanceType>& cat, const vector<int>& its, const Requirements& reqs) {
  if (!HasMinValues(reqs)) return true;
  map<string, set<string>> valuesForKey;
  for (int t : its) {
    for (auto& kv : reqs) {
      if (!kv.second.has_min) continue;
      auto& s = valuesForKey[kv.first];
      auto f = cat[t].reqs.find(kv.first);
      if (f != cat[t].reqs.end()) s.insert(f->second.values.begin(), f->second.values.end());  // Get(key).Values()
    }
    bool ok = true;
    for (auto& kv : valuesForKey)
      if ((int)kv.second.size() < reqs.at(kv.first).min_values) ok = false;
    if (ok) return true;
  }
  return false;
}

struct Counters {
  uint64_t attempts = 0, type_checks = 0, pops = 0, reserved_errors = 0;
};

// UP ReservationManager (scheduling/reservationmanager.go), the design of R:designs/odcr.md:248-256: the scheduler
// counts the simulated NodeClaims that launch into a capacity reservation and stops at its ReservationCapacity.
// capacity starts at the least ReservationCapacity any NodePool's instance types report for the id (two NodePools may
// have listed the reservation at different times); Reserve is idempotent per (hostname, id); Release gives it back.
struct ReservationManager {
  map<string, int64_t> capacity;
  map<string, set<string>> held;  // hostname -> reservation ids
  void Track(const string& id, int64_t cap) {
    auto it = capacity.find(id);
    if (it == capacity.end() || cap < it->second) capacity[id] = cap;
  }
  bool Reserve(const string& host, const string& id) {
    auto& h = held[host];
    if (h.count(id)) return true;
    int64_t& c = capacity.at(id);
    if (c <= 0) return false;
    c--;
    h.insert(id);
    return true;
  }
  void Release(const string& host, const string& id) {
    auto& h = held[host];
    if (h.erase(id)) capacity.at(id)++;
  }
};

static string OfferingResID(const Offering& o) {  // Offering.ReservationID(): the id of a reserved offering
  auto it = o.reqs.find(kLabelResID);
  return it == o.reqs.end() || it->second.values.empty() ? string() : *it->second.values.begin();
}

// filterInstanceTypesByRequirements (UP nodeclaim.go) with relaxMinValues = false.
static bool FilterInstanceTypes(const vector<InstanceType>& cat, const vector<int>& its, const Requirements& reqs,
                                const ResourceList& total, vector<int>* out, Counters* c) {
  out->clear();
  for (int t : its) {
    c->type_checks++;
    const InstanceType& it = cat[t];
    bool compat = Intersects(it.reqs, reqs);
    bool fits = Fits(total, it.allocatable);
    bool hasOffering = false;
    for (auto& o : it.offerings)
      if (o.available && Compatible(reqs, o.reqs, true)) {
        hasOffering = true;
        break;
      }
    if (compat && fits && hasOffering) out->push_back(t);
  }
  if (HasMinValues(reqs) && !SatisfiesMinValues(cat, *out, reqs)) out->clear();
  return !out->empty();
}

struct Scheduler {
  vector<Template> templates;  // ordered by weight desc, name asc
  vector<ExistingNode> existing;
  vector<std::unique_ptr<NodeClaim>> created;  // creation order
  vector<NodeClaim*> newNodeClaims;            // the slice the scheduler sorts
  Topology topology;
  int64_t nodeID = 0;  // hostname placeholder counter (NewNodeClaim)
  Counters counters;
  ReservationManager rm;
  bool strict = false;       // ReservedOfferingModeStrict (the provisioner's DisableReservedCapacityFallback)
  bool reservedErr = false;  // the last NodeClaim.Add failed with a ReservedOfferingError

  // NodeClaim.reserveOfferings (UP nodeclaim.go): every available reserved offering of a remaining type that is
  // compatible with the NodeClaim's new requirements is reserved for its hostname when capacity allows. Strict mode
  // fails the Add when some were compatible but none could be reserved, or when the NodeClaim held reservations and
  // now holds none. A failing call reserved nothing new (the failure means the reserved set is empty).
  bool ReserveOfferings(NodeClaim& n, const Requirements& ncr, const vector<int>& its, set<string>* out) {
    if (rm.capacity.empty()) return true;
    bool compatible = false;
    for (int t : its)
      for (auto& o : (*n.tmpl->catalog)[t].offerings) {
        if (!o.available || *o.reqs.at(kLabelCapacityType).values.begin() != "reserved") continue;
        if (!Compatible(ncr, o.reqs, true)) continue;
        compatible = true;
        const string id = OfferingResID(o);
        if (rm.Reserve(n.hostname, id)) out->insert(id);
      }
    if (strict && out->empty() && (compatible || !n.reserved.empty())) {
      reservedErr = true;
      return false;
    }
    return true;
  }

  // NodeClaim.CanAdd + NodeClaim.Add
  bool NodeClaimAdd(NodeClaim& n, PodState& p) {
    counters.attempts++;
    if (!ToleratesAll(n.tmpl->taints, p.tolerations)) return false;
    if (HostPortsConflict(n.hostPortUsage, p.hostPorts)) return false;
    for (auto& kv : p.requests)  // no remaining option can fit (see NodeClaim.maxalloc)
      if (kv.second > 0 && Get(n.requests, kv.first) + kv.second > n.maxalloc[kv.first]) return false;
    Requirements ncr = n.reqs;
    if (!Compatible(ncr, p.reqs, true)) return false;
    AddAll(ncr, p.reqs);
    Requirements topo;
    if (!topology.AddRequirements(p, ncr, &topo)) return false;
    if (!Compatible(ncr, topo, true)) return false;
    AddAll(ncr, topo);
    ResourceList requests = Merge(n.requests, p.requests);
    vector<int> remaining;
    if (!FilterInstanceTypes(*n.tmpl->catalog, n.options, ncr, requests, &remaining, &counters)) return false;
    set<string> reserved;
    if (!ReserveOfferings(n, ncr, remaining, &reserved)) return false;
    for (auto& id : n.reserved)  // the offerings the narrower NodeClaim no longer reserves go back
      if (!reserved.count(id)) rm.Release(n.hostname, id);
    n.reserved.swap(reserved);
    n.pods.push_back(p.index);
    n.options = std::move(remaining);
    SetMaxAlloc(n);
    n.requests = requests;
    n.reqs = std::move(ncr);
    n.hostPortUsage.insert(n.hostPortUsage.end(), p.hostPorts.begin(), p.hostPorts.end());
    topology.Record(p, n.tmpl->taints, n.reqs, true);
    return true;
  }

  // ExistingNode.CanAdd + ExistingNode.Add
  bool ExistingCanAddAndAdd(ExistingNode& n, PodState& p) {
    counters.attempts++;
    if (!ToleratesAll(n.taints, p.tolerations)) return false;
    if (HostPortsConflict(n.hostPortUsage, p.hostPorts)) return false;
    ResourceList requests = Merge(n.requests, p.requests);
    if (!Fits(requests, n.available)) return false;
    Requirements nr = n.reqs;
    if (!Compatible(nr, p.reqs, false)) return false;
    AddAll(nr, p.reqs);
    Requirements topo;
    if (!topology.AddRequirements(p, nr, &topo)) return false;
    if (!Compatible(nr, topo, false)) return false;
    AddAll(nr, topo);
    n.pods.push_back(p.index);
    n.requests = requests;
    n.reqs = std::move(nr);
    n.hostPortUsage.insert(n.hostPortUsage.end(), p.hostPorts.begin(), p.hostPorts.end());
    topology.Record(p, n.taints, n.reqs, false);
    return true;
  }

  bool anyReservedErr = false;  // addToNewNodeClaim's error for the pod holds a ReservedOfferingError
  bool add(PodState& p) {
    anyReservedErr = false;
    for (auto& n : existing)
      if (ExistingCanAddAndAdd(n, p)) return true;
    struct LS {
      vector<NodeClaim*>& v;
      bool Less(int i, int j) { return v[i]->pods.size() < v[j]->pods.size(); }
      void Swap(int i, int j) { std::swap(v[i], v[j]); }
    } ls{newNodeClaims};
    GoSortSlice(ls, (int)newNodeClaims.size());
    for (NodeClaim* n : newNodeClaims)
      if (NodeClaimAdd(*n, p)) return true;
    if (templates.empty()) return false;
    for (auto& t : templates) {
      vector<int> its = t.options;
      if (t.has_limits) {
        vector<int> f;
        for (int i : its) {
          bool viable = true;
          for (auto& kv : t.remaining)
            if (Get((*t.catalog)[i].capacity, kv.first) > kv.second) viable = false;
          if (viable) f.push_back(i);
        }
        its.swap(f);
        if (its.empty()) continue;
      }
      // NewNodeClaim: template + hostname In {placeholder}, registered with the hostname topologies
      auto nc = std::make_unique<NodeClaim>();
      nc->id = (int)created.size();
      nc->tmpl = &t;
      char hn[64];
      snprintf(hn, sizeof hn, "hostname-placeholder-%04lld", (long long)++nodeID);
      nc->hostname = hn;
      topology.Register(kLabelHostname, nc->hostname);
      nc->reqs = t.reqs;
      Add(nc->reqs, NewRequirement(kLabelHostname, KP_OP_IN, {nc->hostname}, -1));
      nc->options = its;
      SetMaxAlloc(*nc);
      nc->requests = t.daemon;
      reservedErr = false;
      if (!NodeClaimAdd(*nc, p)) {
        anyReservedErr |= reservedErr;
        topology.Unregister(kLabelHostname, nc->hostname);  // NodeClaim.Destroy
        continue;
      }
      if (t.has_limits) {  // subtractMax over the new NodeClaim's InstanceTypeOptions
        ResourceList mx;
        for (int i : nc->options)
          for (auto& kv : (*t.catalog)[i].capacity) {
            auto f = mx.find(kv.first);
            if (f == mx.end() || kv.second > f->second) mx[kv.first] = kv.second;
          }
        for (auto& kv : t.remaining) kv.second -= Get(mx, kv.first);
      }
      newNodeClaims.push_back(nc.get());
      created.push_back(std::move(nc));
      return true;
    }
    return false;
  }
};

}  // namespace oracle

// =============================================================================================
// C API (tests / bench cpu_baseline only)
// =============================================================================================
using namespace oracle;

// Requirements.NodeSelectorRequirements() (Gt, then Lt, then NotIn/Exists, then In/DoesNotExist), keys in
// byte order, values sorted, the hostname placeholder dropped (NodeClaim.FinalizeScheduling).
struct ReqOut {
  std::vector<std::string> keys;
  std::vector<std::vector<std::string>> vals;
  std::vector<std::vector<const char*>> ptrs;
  std::vector<kp_requirement> items;
  void From(const Requirements& r) {
    for (auto& kv : r) {
      if (kv.first == kLabelHostname) continue;
      const Requirement& q = kv.second;
      kp_requirement it;
      memset(&it, 0, sizeof it);
      std::vector<std::string> v;
      if (q.has_gt) {
        it.op = KP_OP_GT;
        v.push_back(std::to_string(q.gt));
      } else if (q.has_lt) {
        it.op = KP_OP_LT;
        v.push_back(std::to_string(q.lt));
      } else if (q.complement) {
        it.op = q.values.empty() ? KP_OP_EXISTS : KP_OP_NOT_IN;
        v.assign(q.values.begin(), q.values.end());
      } else {
        it.op = q.values.empty() ? KP_OP_DOES_NOT_EXIST : KP_OP_IN;
        v.assign(q.values.begin(), q.values.end());
      }
      it.min_values = q.has_min ? q.min_values : -1;
      keys.push_back(kv.first);
      vals.push_back(std::move(v));
      items.push_back(it);
    }
    ptrs.resize(vals.size());
    for (size_t i = 0; i < items.size(); i++) {
      for (auto& x : vals[i]) ptrs[i].push_back(x.c_str());
      items[i].key = keys[i].c_str();
      items[i].values = ptrs[i].data();
      items[i].n_values = (uint32_t)ptrs[i].size();
    }
  }
};

struct kpo_result {
  std::vector<int32_t> placement;
  struct NC {
    uint32_t nodepool;
    std::vector<uint32_t> pods, options;
    uint32_t n_remaining;
    kp_resource_list requests;
    Requirements reqs;                      // final NodeClaim requirements (consolidation needs them)
    const std::vector<InstanceType>* cat = nullptr;
    std::shared_ptr<ReqOut> out;
  };
  std::vector<NC> ncs;
  kp_solve_stats stats;
};

extern "C" {

typedef kp_nodeclaim_info kpo_nodeclaim;

static std::vector<Taint> TaintsFromABI(const kp_taint* t, uint32_t n) {
  std::vector<Taint> v;
  for (uint32_t i = 0; i < n; i++) v.push_back({t[i].key ? t[i].key : "", t[i].value ? t[i].value : "", t[i].effect});
  return v;
}

using Catalogs = std::vector<std::shared_ptr<std::vector<InstanceType>>>;

// Provisioner.NewScheduler + Scheduler.Solve + Results.TruncateInstanceTypes over already-converted catalogues.
static int32_t SolveCore(const Catalogs& cats, const kp_solve_in* in, kpo_result** out) {
  const NamespaceList nsl = NamespacesFromABI(in->namespaces, in->n_namespaces);
  auto t0 = std::chrono::steady_clock::now();
  Scheduler s;
  // NewScheduler: Preferences.ToleratePreferNoSchedule when any NodePool template taint has that effect
  bool toleratePNS = false;
  for (uint32_t i = 0; i < in->n_nodepools; i++)
    for (uint32_t j = 0; j < in->nodepools[i].n_taints; j++)
      toleratePNS = toleratePNS || in->nodepools[i].taints[j].effect == KP_EFFECT_PREFER_NO_SCHEDULE;
  // NewScheduler: templates per NodePool ordered by weight desc, name asc; options pre-filtered by the
  // template requirements with empty requests.
  std::vector<int> order(in->n_nodepools);
  for (uint32_t i = 0; i < in->n_nodepools; i++) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    if (in->nodepools[a].weight != in->nodepools[b].weight) return in->nodepools[a].weight > in->nodepools[b].weight;
    return strcmp(in->nodepools[a].name, in->nodepools[b].name) < 0;
  });
  for (int idx : order) {
    const kp_nodepool& np = in->nodepools[idx];
    if (np.catalog >= in->n_catalogs) return KP_E_INVAL;
    Template t;
    t.nodepool = idx;
    t.name = np.name;
    t.weight = np.weight;
    t.reqs = FromABI(np.requirements);
    AddAll(t.reqs, LabelRequirements(np.labels, np.n_labels));
    Add(t.reqs, NewRequirement(kLabelNodePool, KP_OP_IN, {np.name}, -1));
    t.taints = TaintsFromABI(np.taints, np.n_taints);
    t.catalog = cats[np.catalog].get();
    std::vector<int> all(t.catalog->size());
    for (size_t i = 0; i < all.size(); i++) all[i] = (int)i;
    if (!FilterInstanceTypes(*t.catalog, all, t.reqs, ResourceList{}, &t.options, &s.counters)) continue;
    t.daemon = FromABI(np.daemon_requests);
    t.has_limits = np.limits.present != 0;
    t.remaining = FromABI(np.limits);
    s.templates.push_back(std::move(t));
  }
  // NewReservationManager over the NodePools' instance types
  s.strict = in->reserved_offering_mode == KP_RESERVED_STRICT;
  for (uint32_t i = 0; i < in->n_nodepools; i++)
    for (auto& it : *cats[in->nodepools[i].catalog])
      for (auto& o : it.offerings)
        if (*o.reqs.at(kLabelCapacityType).values.begin() == "reserved") s.rm.Track(OfferingResID(o), o.reservation_capacity);
  // Topology inputs: the node snapshot countDomains reads, the pods bound to it, and buildDomainGroups
  // (NodePool requirements + labels, intersected with each instance type's requirements: In values).
  Topology& topo = s.topology;
  for (uint32_t i = 0; i < in->n_existing; i++) {
    const kp_existing_node& e = in->existing[i];
    NodeView v;
    v.name = e.name ? e.name : "";
    for (uint32_t j = 0; j < e.n_labels; j++) v.labels[e.labels[j].key] = e.labels[j].value ? e.labels[j].value : "";
    v.taints = TaintsFromABI(e.taints, e.n_taints);
    v.reqs = LabelRequirements(e.labels, e.n_labels);
    topo.nodes.push_back(std::move(v));
  }
  for (uint32_t i = 0; i < in->n_bound_pods; i++) {
    const kp_bound_pod& b = in->bound_pods[i];
    if (b.node >= in->n_existing) return KP_E_INVAL;
    BoundPod bp;
    bp.ns = b.namespace_ ? b.namespace_ : "";
    for (uint32_t j = 0; j < b.n_labels; j++) bp.labels[b.labels[j].key] = b.labels[j].value ? b.labels[j].value : "";
    bp.node = (int)b.node;
    for (uint32_t j = 0; j < b.n_anti_affinity; j++) {
      bp.anti.push_back(AntiFromABI(b.anti_affinity[j], bp.ns, nsl));
    }
    topo.bound.push_back(std::move(bp));
  }
  bool anySpread = false;
  for (uint32_t i = 0; i < in->n_shapes; i++)
    anySpread |= in->shapes[i].n_topology_spread > 0 || in->shapes[i].n_required_anti_affinity > 0 ||
                 in->shapes[i].n_preferred_anti_affinity > 0 || in->shapes[i].n_required_affinity > 0 ||
                 in->shapes[i].n_preferred_affinity > 0;
  for (uint32_t i = 0; i < in->n_bound_pods; i++) anySpread |= in->bound_pods[i].n_anti_affinity > 0;
  if (anySpread)
    for (uint32_t i = 0; i < in->n_nodepools; i++) {
      const kp_nodepool& np = in->nodepools[i];
      const auto& cat = *cats[np.catalog];
      if (cat.empty()) continue;
      Requirements base = FromABI(np.requirements);
      AddAll(base, LabelRequirements(np.labels, np.n_labels));
      std::vector<Taint> taints = TaintsFromABI(np.taints, np.n_taints);
      auto insert = [&](const Requirements& r) {
        for (auto& kv : r)
          if (kv.second.Op() == KP_OP_IN)
            for (auto& v : kv.second.values) {
              auto& lst = topo.domainGroups[kv.first][v];
              bool dup = false;
              for (auto& x : lst) {
                bool same = x.size() == taints.size();
                for (size_t k = 0; same && k < x.size(); k++)
                  same = x[k].key == taints[k].key && x[k].value == taints[k].value && x[k].effect == taints[k].effect;
                dup = dup || same;
              }
              if (!dup) lst.push_back(taints);
            }
      };
      for (auto& it : cat) {
        Requirements r = base;
        AddAll(r, it.reqs);
        insert(r);
      }
      insert(base);
    }
  for (uint32_t i = 0; i < in->n_existing; i++) {
    const kp_existing_node& e = in->existing[i];
    ExistingNode n;
    n.index = (int)i;
    n.name = e.name;
    n.initialized = e.initialized != 0;
    n.reqs = LabelRequirements(e.labels, e.n_labels);
    n.taints = TaintsFromABI(e.taints, e.n_taints);
    n.available = FromABI(e.available);
    n.requests = FromABI(e.requests);
    if (!GetHostPorts(e.host_ports, e.n_host_ports, &n.hostPortUsage)) return KP_E_INVAL;
    s.existing.push_back(std::move(n));
  }
  std::stable_sort(s.existing.begin(), s.existing.end(), [](const ExistingNode& a, const ExistingNode& b) {
    if (a.initialized != b.initialized) return a.initialized;
    return a.name < b.name;
  });

  std::vector<PodState> pods(in->n_pods);
  for (uint32_t i = 0; i < in->n_pods; i++) {
    const kp_pod& p = in->pods[i];
    if (p.shape >= in->n_shapes) return KP_E_INVAL;
    const kp_pod_shape& sh = in->shapes[p.shape];
    PodState& ps = pods[i];
    ps.index = (int)i;
    ps.shape = (int)p.shape;
    ps.creation = p.creation_unix;
    ps.uid = p.uid_key;
    if (in->pod_uids) {
      if (!in->pod_uids[i]) return KP_E_INVAL;
      ps.uid_str = in->pod_uids[i];
    }
    ps.requests = FromABI(sh.requests);
    ps.cpu = Get(ps.requests, KP_RES_CPU);
    ps.mem = Get(ps.requests, KP_RES_MEMORY);
    ps.node_selector = LabelRequirements(sh.node_selector, sh.n_node_selector);
    for (uint32_t j = 0; j < sh.n_required_terms; j++) ps.required_terms.push_back(FromABI(sh.required_terms[j]));
    if (sh.n_volume_requirements) {  // UP VolumeTopology.Inject: appended to every required term (one if none)
      const Requirements vol = FromABI(kp_requirements{sh.volume_requirements, sh.n_volume_requirements, 0});
      if (ps.required_terms.empty()) ps.required_terms.push_back(Requirements());
      for (auto& t : ps.required_terms) AddAll(t, vol);
    }
    if (!GetHostPorts(sh.host_ports, sh.n_host_ports, &ps.hostPorts)) return KP_E_INVAL;
    for (uint32_t j = 0; j < sh.n_preferred_terms; j++)
      ps.preferred.push_back({sh.preferred_terms[j].weight, FromABI(sh.preferred_terms[j].preference)});
    for (uint32_t j = 0; j < sh.n_tolerations; j++) {
      const kp_toleration& t = sh.tolerations[j];
      ps.tolerations.push_back({t.key ? t.key : "", t.value ? t.value : "", t.op, t.effect});
    }
    ps.ns = sh.namespace_ ? sh.namespace_ : "";
    for (uint32_t j = 0; j < sh.n_labels; j++) ps.labels[sh.labels[j].key] = sh.labels[j].value ? sh.labels[j].value : "";
    for (uint32_t j = 0; j < sh.n_required_affinity; j++) {
      ps.affRequired.push_back(AntiFromABI(sh.required_affinity[j], ps.ns, nsl));
    }
    for (uint32_t j = 0; j < sh.n_preferred_affinity; j++) {
      ps.affPreferred.push_back(AntiFromABI(sh.preferred_affinity[j], ps.ns, nsl));
    }
    for (uint32_t j = 0; j < sh.n_required_anti_affinity; j++) {
      ps.antiRequired.push_back(AntiFromABI(sh.required_anti_affinity[j], ps.ns, nsl));
    }
    for (uint32_t j = 0; j < sh.n_preferred_anti_affinity; j++) {
      ps.antiPreferred.push_back(AntiFromABI(sh.preferred_anti_affinity[j], ps.ns, nsl));
    }
    for (uint32_t j = 0; j < sh.n_topology_spread; j++) {
      const kp_topology_spread& t = sh.topology_spread[j];
      Spread sp;
      sp.key = t.topology_key ? t.topology_key : "";
      sp.maxSkew = t.max_skew;
      sp.minDomains = t.min_domains > 0 ? t.min_domains : -1;
      sp.when = t.when_unsatisfiable;
      sp.affinityPolicy = t.node_affinity_policy;
      sp.taintsPolicy = t.node_taints_policy;
      sp.sel.nil = t.selector.is_nil != 0;
      for (uint32_t k = 0; k < t.selector.n_match_labels; k++)
        sp.sel.reqs.push_back({t.selector.match_labels[k].key, KP_SEL_IN, {t.selector.match_labels[k].value}});
      for (uint32_t k = 0; k < t.selector.n_match_expressions; k++) {
        const kp_selector_requirement& e = t.selector.match_expressions[k];
        SelReq r{e.key, e.op, {}};
        for (uint32_t v = 0; v < e.n_values; v++) r.values.insert(e.values[v]);
        sp.sel.reqs.push_back(r);
      }
      ps.spreads.push_back(sp);
    }
    ps.reqs = PodRequirements(ps);
    ps.strict = StrictPodRequirements(ps);
  }
  // NewTopology: Update(pod) for every pod of the batch, in input order; then NewExistingNode adds
  // hostname In {HostName()} to each existing node and registers it with the hostname topologies.
  for (auto& ps : pods) topo.Update(ps);
  topo.BuildInverse();  // updateInverseAffinities: after the batch's own groups
  for (auto& n : s.existing) {
    const NodeView& v = topo.nodes[(size_t)n.index];
    auto h = v.labels.find(kLabelHostname);
    const string host = (h == v.labels.end() || h->second.empty()) ? v.name : h->second;
    Add(n.reqs, NewRequirement(kLabelHostname, KP_OP_IN, {host}, -1));
    topo.Register(kLabelHostname, host);
  }

  // Queue (UP queue.go): byCPUAndMemoryDescending, a total order (UID tie-break).
  std::vector<int> q(in->n_pods);
  for (uint32_t i = 0; i < in->n_pods; i++) q[i] = (int)i;
  std::sort(q.begin(), q.end(), [&](int a, int b) {
    const PodState &l = pods[a], &r = pods[b];
    if (l.cpu != r.cpu) return l.cpu > r.cpu;
    if (l.mem != r.mem) return l.mem > r.mem;
    if (l.creation != r.creation) return l.creation < r.creation;
    if (in->pod_uids) return l.uid_str < r.uid_str;  // (UIDs are unique in a cluster)
    return l.uid < r.uid;
  });
  std::vector<int> queue(q.begin(), q.end());
  size_t head = 0;
  std::map<int, size_t> lastLen;
  std::vector<char> errored(in->n_pods, 0);
  for (;;) {
    size_t len = queue.size() - head;
    if (len == 0) break;
    int pi = queue[head];
    auto ll = lastLen.find(pi);
    if (ll != lastLen.end() && ll->second == len) break;
    head++;
    s.counters.pops++;
    PodState& p = pods[pi];
    if (s.add(p)) {
      errored[pi] = 0;
      continue;
    }
    errored[pi] = 1;
    // a ReservedOfferingError is not relaxed: the pod waits for capacity another NodeClaim may release
    if (s.anyReservedErr) s.counters.reserved_errors++;
    bool relaxed = !s.anyReservedErr && Relax(p, toleratePNS);
    queue.push_back(pi);
    if (relaxed) {
      lastLen.clear();
      p.reqs = PodRequirements(p);  // updateCachedPodData
      p.strict = StrictPodRequirements(p);
      s.topology.Update(p);
    } else {
      lastLen[pi] = queue.size() - head;
    }
    // compact occasionally
    if (head > 1024 && head * 2 > queue.size()) {
      queue.erase(queue.begin(), queue.begin() + (long)head);
      head = 0;
    }
  }

  auto* res = new kpo_result();
  res->placement.assign(in->n_pods, -1);
  for (auto& e : s.existing)
    for (int p : e.pods) res->placement[p] = -(2 + e.index);
  // FinalizeScheduling + Results.TruncateInstanceTypes(max): OrderByPrice(reqs) then cut; minValues
  // re-checked on the truncated list, failures turn the NodeClaim's pods into errors.
  for (auto& ncp : s.created) {
    NodeClaim& n = *ncp;
    if (!n.reserved.empty())  // FinalizeScheduling: launch only into the reservations the NodeClaim holds
      Add(n.reqs, NewRequirement(kLabelResID, KP_OP_IN, vector<string>(n.reserved.begin(), n.reserved.end()), -1));
    kpo_result::NC o;
    o.nodepool = (uint32_t)n.tmpl->nodepool;
    o.n_remaining = (uint32_t)n.options.size();
    o.requests = ToABI(n.requests);
    const auto& cat = *n.tmpl->catalog;
    std::vector<std::pair<double, int>> keyed;
    for (int t : n.options) keyed.push_back({CheapestPrice(cat[t], n.reqs), t});
    std::stable_sort(keyed.begin(), keyed.end(), [&](const std::pair<double, int>& a, const std::pair<double, int>& b) {
      if (a.first == b.first) return cat[a.second].name < cat[b.second].name;
      return a.first < b.first;
    });
    std::vector<int> trunc;
    size_t lim = in->max_instance_types ? std::min<size_t>(keyed.size(), in->max_instance_types) : keyed.size();
    for (size_t i = 0; i < lim; i++) trunc.push_back(keyed[i].second);
    bool ok = !HasMinValues(n.reqs) || SatisfiesMinValues(cat, trunc, n.reqs);
    o.reqs = n.reqs;
    o.cat = &cat;
    o.out = std::make_shared<ReqOut>();
    o.out->From(n.reqs);
    if (ok) {
      for (int t : trunc) o.options.push_back((uint32_t)t);
      for (int p : n.pods) {
        o.pods.push_back((uint32_t)p);
        res->placement[p] = n.id;
      }
    } else {
      for (int p : n.pods) o.pods.push_back((uint32_t)p);  // pods listed, placement stays -1
    }
    res->ncs.push_back(std::move(o));
  }
  (void)errored;
  memset(&res->stats, 0, sizeof(res->stats));
  res->stats.attempts = s.counters.attempts;
  res->stats.pops = s.counters.pops;
  res->stats.reserved_offering_errors = s.counters.reserved_errors;
  res->stats.bytes_algorithmic = s.counters.type_checks;  // type rows visited (SURVEY §8d counter)
  res->stats.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = res;
  return KP_OK;
}

int32_t kpo_solve(const kp_solve_in* in, kpo_result** out) {
  if (!in || !out || (!in->catalog_descs && in->n_catalogs)) return KP_E_INVAL;
  Catalogs cats;
  for (uint32_t i = 0; i < in->n_catalogs; i++) cats.push_back(CatalogFromABI(in->catalog_descs[i]));
  return SolveCore(cats, in, out);
}


// ---- disruption: computeConsolidation over candidate subsets -------------
// Offerings.Compatible(NewLabelRequirements(node labels)).Cheapest().Price (getCandidatePrices /
// filterOutSameType); false when no offering is label-compatible.
static bool CandidatePrice(const InstanceType& it, const Requirements& labels, double* price) {
  bool any = false;
  double p = 0;
  for (auto& o : it.offerings)
    if (Compatible(labels, o.reqs, true)) {
      if (!any || o.price < p) p = o.price;
      any = true;
    }
  *price = p;
  return any;
}
// Offerings.Available().WorstLaunchPrice(reqs): capacity types in precedence reserved, spot, on-demand;
// the most expensive compatible available offering of the first capacity type that has one.
static double WorstLaunchPrice(const InstanceType& it, const Requirements& reqs, bool spot_only = false) {
  for (const char* ct : {"reserved", "spot", "on-demand"}) {
    if (spot_only && std::string(ct) != "spot") continue;  // requirements narrowed to capacity-type In {spot}
    bool any = false;
    double mx = 0;
    for (auto& o : it.offerings) {
      if (!o.available || !Compatible(reqs, o.reqs, true)) continue;
      auto f = o.reqs.find(kLabelCapacityType);
      if (f == o.reqs.end() || !Has(f->second, ct)) continue;
      if (!any || o.price > mx) mx = o.price;
      any = true;
    }
    if (any) return mx;
  }
  return std::numeric_limits<double>::max();
}

int32_t kpo_simulate_batch(const kp_cluster* cl, const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                           int32_t multi_node, kp_sim_result* out, kp_solve_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!cl || !offsets || !out || (!cl->catalog_descs && cl->n_catalogs)) return KP_E_INVAL;
  Catalogs cats;
  for (uint32_t i = 0; i < cl->n_catalogs; i++) cats.push_back(CatalogFromABI(cl->catalog_descs[i]));
  std::vector<Requirements> nodeLabels(cl->n_nodes);
  for (uint32_t i = 0; i < cl->n_nodes; i++) nodeLabels[i] = LabelRequirements(cl->nodes[i].node.labels, cl->nodes[i].node.n_labels);
  uint64_t attempts = 0;
  std::vector<char> inS(cl->n_nodes, 0);
  for (uint32_t s = 0; s < n_subsets; s++) {
    kp_sim_result& r = out[s];
    memset(&r, 0, sizeof r);
    std::vector<uint32_t> cand(nodes + offsets[s], nodes + offsets[s + 1]);
    for (uint32_t c : cand) {
      if (cl->nodes[c].deleting) return KP_E_INVAL;  // candidates never include nodes already being deleted
      inS[c] = 1;
    }
    // SimulateScheduling: the pending pods, the pods of the deleting nodes and of the candidates; every node that
    // is neither a candidate nor deleting is an existing node. kind: 0 candidate pod, 1 deleting-node pod, 2 pending
    std::vector<kp_existing_node> ex;
    std::vector<uint32_t> exIdx;
    for (uint32_t i = 0; i < cl->n_nodes; i++)
      if (!inS[i] && !cl->nodes[i].deleting) {
        ex.push_back(cl->nodes[i].node);
        exIdx.push_back(i);
      }
    std::vector<kp_pod> pods;
    std::vector<int> kind;
    std::vector<const char*> uids;
    auto add = [&](uint32_t p, int k) {
      pods.push_back(cl->pods[p]);
      kind.push_back(k);
      if (cl->pod_uids) uids.push_back(cl->pod_uids[p]);
    };
    for (uint32_t j = 0; j < cl->n_pending; j++) add(cl->pending_pods[j], 2);
    for (uint32_t i = 0; i < cl->n_nodes; i++)
      if (cl->nodes[i].deleting)
        for (uint32_t j = 0; j < cl->nodes[i].n_pods; j++) add(cl->nodes[i].pods[j], 1);
    for (uint32_t c : cand)
      for (uint32_t j = 0; j < cl->nodes[c].n_pods; j++) add(cl->nodes[c].pods[j], 0);
    for (uint32_t c : cand) inS[c] = 0;
    // Topology.countDomains lists every pod bound to a node except the pods being scheduled: the pods of the
    // remaining nodes are the bound pods (their shape's namespace and labels)
    std::vector<kp_bound_pod> bound;
    for (size_t e = 0; e < exIdx.size(); e++) {
      const kp_cluster_node& n = cl->nodes[exIdx[e]];
      for (uint32_t j = 0; j < n.n_pods; j++) {
        const kp_pod_shape& sh = cl->shapes[cl->pods[n.pods[j]].shape];
        bound.push_back({sh.namespace_, sh.labels, sh.n_labels, (uint32_t)e, sh.required_anti_affinity,
                         sh.n_required_anti_affinity, 0});
      }
    }
    r.n_pods = (uint32_t)pods.size();
    kp_solve_in in;
    memset(&in, 0, sizeof in);
    in.n_catalogs = cl->n_catalogs;
    in.catalog_descs = cl->catalog_descs;
    in.n_nodepools = cl->n_nodepools;
    in.nodepools = cl->nodepools;
    in.existing = ex.data();
    in.n_existing = (uint32_t)ex.size();
    in.n_shapes = cl->n_shapes;
    in.shapes = cl->shapes;
    in.pods = pods.data();
    in.n_pods = (uint32_t)pods.size();
    in.max_instance_types = 100;
    in.bound_pods = bound.data();
    in.n_bound_pods = (uint32_t)bound.size();
    in.namespaces = cl->namespaces;
    in.n_namespaces = cl->n_namespaces;
    in.pod_uids = cl->pod_uids ? uids.data() : nullptr;
    // SimulateScheduling builds its scheduler with DisableReservedCapacityFallback: strict reservations
    in.reserved_offering_mode = KP_RESERVED_STRICT;
    kpo_result* res = nullptr;
    int32_t rc = SolveCore(cats, &in, &res);
    if (rc) return rc;
    std::unique_ptr<kpo_result> guard(res);
    attempts += res->stats.attempts;
    // AllNonPendingPodsScheduled: every pod that was not pending scheduled; a candidate pod on an uninitialized
    // node is SimulateScheduling's UninitializedNodeError (pods of deleting nodes are exempt)
    bool all = true;
    for (size_t p = 0; p < res->placement.size(); p++) {
      const int32_t pl = res->placement[p];
      if (kind[p] == 2) continue;
      if (pl == -1) all = false;
      else if (kind[p] == 0 && pl <= -2 && !ex[(size_t)(-2 - pl)].initialized) all = false;
    }
    double candPrice = 0;
    bool priced = true;
    for (uint32_t c : cand) {
      const kp_cluster_node& n = cl->nodes[c];
      double p;
      if (!CandidatePrice((*cats[n.catalog])[n.instance_type], nodeLabels[c], &p)) priced = false;
      candPrice += p;
    }
    r.candidate_price = priced ? candPrice : 0;
    if (!all) continue;  // no-op
    if (res->ncs.empty()) {
      r.decision = KP_DECISION_DELETE;
      r.savings = r.candidate_price;
      continue;
    }
    if (res->ncs.size() != 1 || !priced) continue;
    const auto& nc = res->ncs[0];
    const auto& cat = *nc.cat;
    bool allSpot = true;
    for (uint32_t c : cand) {
      auto f = nodeLabels[c].find(kLabelCapacityType);
      if (f == nodeLabels[c].end() || f->second.complement || !f->second.values.count("spot")) allSpot = false;
    }
    auto ctr = nc.reqs.find(kLabelCapacityType);
    const bool ncSpot = ctr == nc.reqs.end() || Has(ctr->second, "spot");
    // spot-to-spot consolidation (every candidate spot, the replacement may launch spot): only with the feature
    // gate; the replacement's requirements are narrowed to capacity-type In {spot} (its options keep only spot
    // offerings), and a single candidate needs MinInstanceTypesForSpotToSpotConsolidation = 15 cheaper options,
    // after which the launch keeps the cheapest 15 (100 with minValues) — disruption.md:110-128
    const bool s2s = allSpot && ncSpot;
    if (s2s && !cl->spot_to_spot) continue;
    std::vector<int> kept;
    for (uint32_t t : nc.options)
      if (WorstLaunchPrice(cat[t], nc.reqs, s2s) < candPrice) kept.push_back((int)t);
    if (HasMinValues(nc.reqs) && !SatisfiesMinValues(cat, kept, nc.reqs)) continue;
    if (kept.empty()) continue;
    if (multi_node) {  // filterOutSameType
      std::map<std::string, double> prices;
      for (uint32_t c : cand) {
        const kp_cluster_node& n = cl->nodes[c];
        const InstanceType& it = (*cats[n.catalog])[n.instance_type];
        double p;
        if (!CandidatePrice(it, nodeLabels[c], &p)) continue;
        auto f = prices.find(it.name);
        if (f == prices.end() || p < f->second) prices[it.name] = p;
      }
      double maxPrice = std::numeric_limits<double>::max();
      for (int t : kept) {
        auto f = prices.find(cat[t].name);
        if (f != prices.end() && f->second < maxPrice) maxPrice = f->second;
      }
      std::vector<int> k2;
      for (int t : kept)
        if (WorstLaunchPrice(cat[t], nc.reqs, s2s) < maxPrice) k2.push_back(t);
      if (HasMinValues(nc.reqs) && !SatisfiesMinValues(cat, k2, nc.reqs)) continue;
      kept.swap(k2);
      if (kept.empty()) continue;
    }
    if (s2s && cand.size() == 1) {
      if (kept.size() < 15) continue;
      kept.resize(std::min<size_t>(kept.size(), HasMinValues(nc.reqs) ? 100 : 15));  // kept is in price order
    }
    double best = std::numeric_limits<double>::max();
    for (int t : kept) best = std::min(best, WorstLaunchPrice(cat[t], nc.reqs, s2s));
    r.decision = KP_DECISION_REPLACE;
    r.replacement_nodepool = nc.nodepool;
    r.replacement_price = best;
    r.savings = candPrice - best;
    r.n_options = (uint32_t)kept.size();
  }
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->attempts = attempts;
    stats->host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return KP_OK;
}

uint32_t kpo_result_nodeclaim_count(const kpo_result* r) { return (uint32_t)r->ncs.size(); }
int32_t kpo_result_pod_placements(const kpo_result* r, int32_t* out, uint32_t n) {
  if (n != r->placement.size()) return KP_E_INVAL;
  memcpy(out, r->placement.data(), n * sizeof(int32_t));
  return KP_OK;
}
int32_t kpo_result_nodeclaim(const kpo_result* r, uint32_t i, kpo_nodeclaim* out) {
  if (i >= r->ncs.size()) return KP_E_INVAL;
  const auto& n = r->ncs[i];
  out->nodepool = n.nodepool;
  out->n_pods = (uint32_t)n.pods.size();
  out->n_remaining = n.n_remaining;
  out->n_options = (uint32_t)n.options.size();
  out->pods = n.pods.data();
  out->options = n.options.data();
  out->requests = n.requests;
  out->requirements.items = n.out ? n.out->items.data() : nullptr;
  out->requirements.n = n.out ? (uint32_t)n.out->items.size() : 0;
  out->requirements.reserved_ = 0;
  return KP_OK;
}
int32_t kpo_result_stats(const kpo_result* r, kp_solve_stats* out) {
  *out = r->stats;
  return KP_OK;
}
void kpo_result_destroy(kpo_result* r) { delete r; }

// CompatibleAvailableFilter (R:filter.go:39-64) for one query; out_kept[t] = 1 when kept.
// out_cheapest[t] = cheapest compatible available price (+inf when none).
int32_t kpo_filter_compatible_available(const kp_catalog_desc* cat, const kp_feasibility_query* q, uint8_t* out_kept,
                                        double* out_cheapest) {
  auto types = CatalogFromABI(*cat);
  Requirements reqs = FromABI(q->requirements);
  ResourceList requests = FromABI(q->requests);
  for (size_t t = 0; t < types->size(); t++) {
    const InstanceType& it = (*types)[t];
    bool kept = Compatible(reqs, it.reqs, true) && Fits(requests, it.allocatable) && HasCompatibleAvailable(it, reqs);
    out_kept[t] = kept ? 1 : 0;
    if (out_cheapest) {
      bool any = false;
      double p = INFINITY;
      for (auto& o : it.offerings)
        if (o.available && Compatible(reqs, o.reqs, true)) {
          if (!any || o.price < p) p = o.price;
          any = true;
        }
      out_cheapest[t] = p;
    }
  }
  return KP_OK;
}

// SpotInstanceFilter (R:filter.go:328-386); reserved offerings are not representable in ABI v1.
int32_t kpo_filter_spot(const kp_catalog_desc* cat, const kp_requirements* req, uint8_t* out_kept) {
  auto types = CatalogFromABI(*cat);
  Requirements reqs = FromABI(*req);
  for (size_t t = 0; t < types->size(); t++) out_kept[t] = 1;
  if (HasMinValues(reqs)) return KP_OK;
  // Requirements.Get(key) of an absent key is Exists: Has() every value
  auto ct = reqs.find(kLabelCapacityType);
  if (ct != reqs.end() && (!Has(ct->second, "on-demand") || !Has(ct->second, "spot"))) return KP_OK;
  double cheapestOD = std::numeric_limits<double>::max();
  bool hasSpot = false, hasOD = false;
  auto capType = [](const Offering& o) { return *o.reqs.at(kLabelCapacityType).values.begin(); };
  for (auto& it : *types)
    for (auto& o : it.offerings) {
      if (!Compatible(reqs, o.reqs, true) || !o.available) continue;
      std::string c = capType(o);
      if (c == "on-demand") {
        hasOD = true;
        if (o.price < cheapestOD) cheapestOD = o.price;
      } else if (c == "spot") {
        hasSpot = true;
      }
    }
  if (!hasOD || !hasSpot) return KP_OK;
  for (size_t t = 0; t < types->size(); t++) {
    bool hasSpotOffering = false, keep = false;
    for (auto& o : (*types)[t].offerings) {
      if (!Compatible(reqs, o.reqs, true) || !o.available) continue;
      std::string c = capType(o);
      if (c == "reserved") {
        keep = true;
        break;
      }
      if (c == "spot") {
        hasSpotOffering = true;
        if (o.price <= cheapestOD) {
          keep = true;
          break;
        }
      }
    }
    out_kept[t] = (keep || !hasSpotOffering) ? 1 : 0;
  }
  return KP_OK;
}

// ExoticInstanceTypeFilter (R:filter.go:279-318)
int32_t kpo_filter_exotic(const kp_catalog_desc* cat, const kp_requirements* req, uint8_t* out_kept) {
  auto types = CatalogFromABI(*cat);
  Requirements reqs = FromABI(*req);
  size_t n = types->size();
  for (size_t t = 0; t < n; t++) out_kept[t] = 1;
  if (HasMinValues(reqs)) return KP_OK;
  std::vector<uint8_t> generic(n, 0);
  size_t ng = 0;
  for (size_t t = 0; t < n; t++) {
    const InstanceType& it = (*types)[t];
    bool exotic = false;
    auto sz = it.reqs.find(AWSL("instance-size"));
    if (sz != it.reqs.end() && !sz->second.complement)
      for (auto& v : sz->second.values)
        if (v.find("metal") != std::string::npos) exotic = true;
    for (int r : {KP_RES_NEURON, KP_RES_NEURONCORE, KP_RES_AMD_GPU, KP_RES_NVIDIA_GPU, KP_RES_GAUDI})
      if (Get(it.capacity, r) != 0) exotic = true;
    generic[t] = !exotic;
    ng += !exotic;
  }
  if (ng == 0) return KP_OK;
  for (size_t t = 0; t < n; t++) out_kept[t] = generic[t];
  return KP_OK;
}

// ---- launch-side selection: instance.DefaultProvider.Create (R:pkg/providers/instance/instance.go:117-125) ----
// Requirements.Get(key).Has(v): an absent key is Exists (every value).
static bool ReqHas(const Requirements& r, const string& key, const string& v) {
  auto f = r.find(key);
  return f == r.end() || Has(f->second, v);
}
static string OfferingCapType(const Offering& o) { return *o.reqs.at(kLabelCapacityType).values.begin(); }
static string OfferingZone(const Offering& o) {
  auto f = o.reqs.find(kLabelZone);
  return f == o.reqs.end() || f->second.values.empty() ? string() : *f->second.values.begin();
}
static bool IsExotic(const InstanceType& it) {  // R:filter.go:295-310
  auto sz = it.reqs.find(AWSL("instance-size"));
  if (sz != it.reqs.end() && !sz->second.complement)
    for (auto& v : sz->second.values)
      if (v.find("metal") != std::string::npos) return true;
  for (int r : {KP_RES_NEURON, KP_RES_NEURONCORE, KP_RES_AMD_GPU, KP_RES_NVIDIA_GPU, KP_RES_GAUDI})
    if (Get(it.capacity, r) != 0) return true;
  return false;
}

// A launch's working list: each instance type with its current offering list (indices into the catalogue's
// offerings). The reservation filters replace a type's offering slice (R:filter.go:107-116, 196-200, 253-257);
// everything after them reads the replaced slices. Where the reference returns map values (lo.Values: random
// order) this keeps list / offering order.
struct WorkType {
  int t;
  vector<int> offs;
};
static string OfferingResType(const Offering& o) {  // Requirements.Get(capacity-reservation-type).Any(); "" for DNE
  auto f = o.reqs.find(kLabelResType);
  return f == o.reqs.end() || f->second.complement || f->second.values.empty() ? string() : *f->second.values.begin();
}
static int ResTypeIndex(const string& rt) {  // v1.CapacityReservationType("").Values() order = priority order
  return rt == "default" ? 0 : rt == "capacity-block" ? 1 : -1;
}

// CapacityReservationTypeFilter (R:filter.go:66-144): the partition (default / capacity-block) holding the
// cheapest available compatible reserved offering (ties: priority default < capacity-block); its types keep only
// their reserved offerings of that type, the rest are rejected; an empty selected partition keeps everything.
// A reserved offering without a reservation type (the reference panics) belongs to no partition.
static void FilterCapacityReservationType(const vector<InstanceType>& C, const Requirements& reqs, vector<WorkType>& W) {
  if (!ReqHas(reqs, kLabelCapacityType, "reserved")) return;
  double cheapest[2] = {std::numeric_limits<double>::max(), std::numeric_limits<double>::max()};
  vector<char> member[2] = {vector<char>(W.size(), 0), vector<char>(W.size(), 0)};
  for (size_t i = 0; i < W.size(); i++)
    for (int oi : W[i].offs) {
      const Offering& o = C[W[i].t].offerings[oi];
      if (!o.available || !Compatible(reqs, o.reqs, true) || OfferingCapType(o) != "reserved") continue;
      const int p = ResTypeIndex(OfferingResType(o));
      if (p < 0) continue;
      if (o.price < cheapest[p]) cheapest[p] = o.price;
      member[p][i] = 1;
    }
  const int sel = cheapest[1] < cheapest[0] ? 1 : 0;
  vector<WorkType> kept;
  for (size_t i = 0; i < W.size(); i++)
    if (member[sel][i]) {
      WorkType w{W[i].t, {}};
      for (int oi : W[i].offs) {
        const Offering& o = C[W[i].t].offerings[oi];
        if (OfferingCapType(o) == "reserved" && ResTypeIndex(OfferingResType(o)) == sel) w.offs.push_back(oi);
      }
      kept.push_back(std::move(w));
    }
  if (!kept.empty()) W = std::move(kept);
}

// CapacityBlockFilter (R:filter.go:146-225): applies when the first offering of the first type carries the
// capacity-block reservation type (every offering carries the key: DoesNotExist on non-reserved ones,
// R:offering.go:136-137); keeps the single type whose cheapest capacity-block offering (any availability) is the
// cheapest, with only that offering.
static void FilterCapacityBlock(const vector<InstanceType>& C, const Requirements& reqs, vector<WorkType>& W) {
  if (!ReqHas(reqs, kLabelCapacityType, "reserved")) return;
  bool should = false;
  for (auto& w : W)
    if (!w.offs.empty()) {
      should = ResTypeIndex(OfferingResType(C[w.t].offerings[w.offs[0]])) == 1;
      break;
    }
  if (!should) return;
  int sel_w = -1;
  double sel_price = 0;
  for (size_t i = 0; i < W.size(); i++) {
    int so = -1;
    for (int oi : W[i].offs) {
      const Offering& o = C[W[i].t].offerings[oi];
      if (OfferingCapType(o) != "reserved" || ResTypeIndex(OfferingResType(o)) != 1) continue;
      if (so < 0 || C[W[i].t].offerings[so].price > o.price) so = oi;
    }
    if (so >= 0 && (sel_w < 0 || sel_price > C[W[i].t].offerings[so].price)) {
      W[i].offs = {so};
      sel_w = (int)i;
      sel_price = C[W[i].t].offerings[so].price;
    }
  }
  if (sel_w < 0) return;  // no reserved capacity-block offering at all (the reference dereferences nil here)
  W = {W[sel_w]};
}

// ReservedOfferingFilter (R:filter.go:227-274): per type, one available compatible reserved offering per zone (the
// greatest ReservationCapacity, the first on ties); types without one are rejected unless that rejects all.
static void FilterReservedOffering(const vector<InstanceType>& C, const Requirements& reqs, vector<WorkType>& W) {
  if (!ReqHas(reqs, kLabelCapacityType, "reserved")) return;
  vector<WorkType> kept;
  for (auto& w : W) {
    vector<std::pair<string, int>> zonal;  // zone -> offering, in first-seen order
    for (int oi : w.offs) {
      const Offering& o = C[w.t].offerings[oi];
      if (!o.available || !Compatible(reqs, o.reqs, true) || OfferingCapType(o) != "reserved") continue;
      const string z = OfferingZone(o);
      auto f = std::find_if(zonal.begin(), zonal.end(), [&](const std::pair<string, int>& e) { return e.first == z; });
      if (f == zonal.end()) zonal.push_back({z, oi});
      else if (o.reservation_capacity > C[w.t].offerings[f->second].reservation_capacity) f->second = oi;
    }
    if (zonal.empty()) continue;
    WorkType k{w.t, {}};
    for (auto& e : zonal) k.offs.push_back(e.second);
    std::sort(k.offs.begin(), k.offs.end());
    kept.push_back(std::move(k));
  }
  if (!kept.empty()) W = std::move(kept);
}

static bool WorkHasCompatibleAvailable(const vector<InstanceType>& C, const WorkType& w, const Requirements& reqs,
                                       const char* ct = nullptr) {
  for (int oi : w.offs) {
    const Offering& o = C[w.t].offerings[oi];
    if (o.available && Compatible(reqs, o.reqs, true) && (!ct || OfferingCapType(o) == ct)) return true;
  }
  return false;
}
static double WorkCheapest(const vector<InstanceType>& C, const WorkType& w, const Requirements& reqs) {
  double p = std::numeric_limits<double>::max();
  for (int oi : w.offs) {
    const Offering& o = C[w.t].offerings[oi];
    if (o.available && Compatible(reqs, o.reqs, true) && o.price < p) p = o.price;
  }
  return p;
}

// One reservation filter over the whole catalogue (in order, every offering): which 0 CapacityReservationType,
// 1 CapacityBlock, 2 ReservedOffering. out_kept[t]: the type is in the returned list; out_offering_kept[flat
// offering index]: the offering is in its type's (replaced) slice. Pinned by R:filter_test.go:130-396.
int32_t kpo_filter_reservation(const kp_catalog_desc* cat, const kp_requirements* req, int32_t which, uint8_t* out_kept,
                               uint8_t* out_offering_kept) {
  auto types = CatalogFromABI(*cat);
  const vector<InstanceType>& C = *types;
  Requirements reqs = FromABI(*req);
  vector<WorkType> W;
  for (size_t t = 0; t < C.size(); t++) {
    WorkType w{(int)t, {}};
    for (size_t j = 0; j < C[t].offerings.size(); j++) w.offs.push_back((int)j);
    W.push_back(std::move(w));
  }
  if (which == 0) FilterCapacityReservationType(C, reqs, W);
  else if (which == 1) FilterCapacityBlock(C, reqs, W);
  else if (which == 2) FilterReservedOffering(C, reqs, W);
  else return KP_E_INVAL;
  vector<size_t> first(C.size() + 1, 0);
  for (size_t t = 0; t < C.size(); t++) first[t + 1] = first[t] + C[t].offerings.size();
  std::fill(out_kept, out_kept + C.size(), 0);
  std::fill(out_offering_kept, out_offering_kept + first[C.size()], 0);
  for (auto& w : W) {
    out_kept[w.t] = 1;
    for (int oi : w.offs) out_offering_kept[first[w.t] + oi] = 1;
  }
  return KP_OK;
}

// filterInstanceTypes (R:instance.go:242-270) + getCapacityType (:504-518) + checkODFallback (:336-355) +
// getOverrides (:392-439) + getCapacityReservationType (:520-530) for one NodeClaim.
int32_t kpo_launch_select(const kp_catalog_desc* cat, const kp_launch_request* req, const char* const* zones,
                          uint32_t n_zones, uint32_t max_types, kp_launch_result* out, uint32_t* out_types,
                          uint32_t* out_overrides) {
  auto types = CatalogFromABI(*cat);
  const vector<InstanceType>& C = *types;
  Requirements reqs = FromABI(req->requirements);
  ResourceList requests = FromABI(req->requests);
  *out = kp_launch_result{};
  out->failed_filter = -1;
  out->reservation_type = -1;
  vector<WorkType> W;
  for (uint32_t i = 0; i < req->n_instance_types; i++) {
    if (req->instance_types[i] >= C.size()) return KP_E_INVAL;
    const int t = (int)req->instance_types[i];
    // CompatibleAvailableFilter (R:filter.go:51-63)
    if (!(Compatible(reqs, C[t].reqs, true) && Fits(requests, C[t].allocatable) && HasCompatibleAvailable(C[t], reqs)))
      continue;
    WorkType w{t, {}};
    for (size_t j = 0; j < C[t].offerings.size(); j++) w.offs.push_back((int)j);
    W.push_back(std::move(w));
  }
  out->n_compatible = (uint32_t)W.size();
  if (W.empty()) {
    out->status = KP_LAUNCH_INSUFFICIENT_CAPACITY;
    out->failed_filter = KP_FILTER_COMPATIBLE_AVAILABLE;
    return KP_OK;
  }
  // the reservation filters never empty the list (each keeps its input rather than nothing)
  size_t n0 = W.size();
  FilterCapacityReservationType(C, reqs, W);
  out->rejected_reservation = (uint32_t)(n0 - W.size());
  n0 = W.size();
  FilterCapacityBlock(C, reqs, W);
  out->rejected_reservation += (uint32_t)(n0 - W.size());
  n0 = W.size();
  FilterReservedOffering(C, reqs, W);
  out->rejected_reservation += (uint32_t)(n0 - W.size());
  const bool hasMin = HasMinValues(reqs);
  // ExoticInstanceTypeFilter (R:filter.go:289-314): keep the generic types if any
  if (!hasMin) {
    vector<WorkType> generic;
    for (auto& w : W)
      if (!IsExotic(C[w.t])) generic.push_back(w);
    if (!generic.empty()) {
      out->rejected_exotic = (uint32_t)(W.size() - generic.size());
      W = std::move(generic);
    }
  }
  // SpotInstanceFilter (R:filter.go:342-382)
  if (!hasMin && ReqHas(reqs, kLabelCapacityType, "on-demand") && ReqHas(reqs, kLabelCapacityType, "spot")) {
    double cheapestOD = std::numeric_limits<double>::max();
    bool hasSpot = false, hasOD = false;
    for (auto& w : W)
      for (int oi : w.offs) {
        const Offering& o = C[w.t].offerings[oi];
        if (!Compatible(reqs, o.reqs, true) || !o.available) continue;
        const string c = OfferingCapType(o);
        if (c == "on-demand") {
          hasOD = true;
          if (o.price < cheapestOD) cheapestOD = o.price;
        } else if (c == "spot") {
          hasSpot = true;
        }
      }
    if (hasOD && hasSpot) {
      vector<WorkType> k2;
      for (auto& w : W) {
        bool hasSpotOffering = false, keep = false;
        for (int oi : w.offs) {
          const Offering& o = C[w.t].offerings[oi];
          if (!Compatible(reqs, o.reqs, true) || !o.available) continue;
          const string c = OfferingCapType(o);
          if (c == "reserved") {  // modelled as free: always kept (R:filter.go:368-371)
            keep = true;
            break;
          }
          if (c == "spot") {
            hasSpotOffering = true;
            if (o.price <= cheapestOD) {
              keep = true;
              break;
            }
          }
        }
        if (keep || !hasSpotOffering) k2.push_back(w);
      }
      out->rejected_spot = (uint32_t)(W.size() - k2.size());
      if (k2.empty()) {
        out->status = KP_LAUNCH_INSUFFICIENT_CAPACITY;
        out->failed_filter = KP_FILTER_SPOT;
        return KP_OK;
      }
      W = std::move(k2);
    }
  }
  // InstanceTypes.Truncate(reqs, maxInstanceTypes): OrderByPrice (cheapest available compatible, then name)
  std::stable_sort(W.begin(), W.end(), [&](const WorkType& a, const WorkType& b) {
    const double pa = WorkCheapest(C, a, reqs), pb = WorkCheapest(C, b, reqs);
    if (pa != pb) return pa < pb;
    return C[a.t].name < C[b.t].name;
  });
  if (max_types && W.size() > max_types) W.resize(max_types);
  if (hasMin) {
    vector<int> its;
    for (auto& w : W) its.push_back(w.t);
    if (!SatisfiesMinValues(C, its, reqs)) {
      out->status = KP_LAUNCH_MINVALUES;
      return KP_OK;
    }
  }
  // getCapacityType: reserved, then spot, when the requirements allow it and a remaining type has an available
  // offering compatible with the requirements pinned to it
  int ct = 0;
  const char* ct_names[3] = {"on-demand", "spot", "reserved"};
  for (int cand : {2, 1}) {
    if (!ReqHas(reqs, kLabelCapacityType, ct_names[cand])) continue;
    Requirements r2 = reqs;
    r2[kLabelCapacityType] = NewRequirement(kLabelCapacityType, KP_OP_IN, {ct_names[cand]}, -1);
    for (auto& w : W)
      if (WorkHasCompatibleAvailable(C, w, r2)) {
        ct = cand;
        break;
      }
    if (ct) break;
  }
  out->capacity_type = ct;
  out->od_fallback_warning = ct == 0 && ReqHas(reqs, kLabelCapacityType, "spot") && W.size() < 5;
  if (ct == 2)  // getCapacityReservationType: the first offering (of the first type) carrying the key
    for (auto& w : W)
      if (!w.offs.empty()) {
        out->reservation_type = ResTypeIndex(OfferingResType(C[w.t].offerings[w.offs[0]]));
        break;
      }
  // getOverrides with the capacity type pinned; zonalSubnets = subnet_zones
  Requirements r3 = reqs;
  r3[kLabelCapacityType] = NewRequirement(kLabelCapacityType, KP_OP_IN, {ct_names[ct]}, -1);
  uint32_t no = 0;
  for (size_t i = 0; i < W.size(); i++) {
    out_types[i] = (uint32_t)W[i].t;
    for (int oi : W[i].offs) {
      const Offering& o = C[W[i].t].offerings[oi];
      if (!o.available || !Compatible(r3, o.reqs, true)) continue;
      const string z = OfferingZone(o);
      for (uint32_t zi = 0; zi < n_zones; zi++)
        if (z == zones[zi]) {
          out_overrides[no++] = ((uint32_t)W[i].t << 8) | zi;
          break;
        }
    }
  }
  out->n_types = (uint32_t)W.size();
  out->n_overrides = no;
  return KP_OK;
}

// Requirements algebra probe for tests: Compatible(a, b, allowUndefinedWellKnown) and Intersects(a, b).
int32_t kpo_requirements_compatible(const kp_requirements* a, const kp_requirements* b, int32_t allow_wk) {
  return Compatible(FromABI(*a), FromABI(*b), allow_wk != 0) ? 1 : 0;
}
int32_t kpo_requirements_intersects(const kp_requirements* a, const kp_requirements* b) {
  return Intersects(FromABI(*a), FromABI(*b)) ? 1 : 0;
}

// ---- catalogue: NewInstanceType (R:types.go:123-598) per AMI family ------------------------------
// FeatureFlags: DefaultFamily (AL2023, AL2, Custom) R:pkg/providers/amifamily/resolver.go:110-117, Bottlerocket
// bottlerocket.go:126-132, Windows windows.go:101-108; default ephemeral volume (no blockDeviceMappings): the family's
// EphemeralBlockDevice in its DefaultBlockDeviceMappings, else DefaultEBS (20Gi) (R:types.go:350-388).
struct AMIFamilyFlags {
  bool UsesENILimitedMemoryOverhead, PodsPerCoreEnabled, EvictionSoftEnabled, SupportsENILimitedPodDensity, Windows;
  int64_t EphemeralGi;
};
static AMIFamilyFlags FamilyOf(const kp_nodeclass* nc) {
  switch (nc ? nc->ami_family : KP_AMI_AL2023) {
    case KP_AMI_BOTTLEROCKET:
      return {false, false, false, true, false, 20};  // /dev/xvdb: DefaultEBS
    case KP_AMI_WINDOWS2019:
    case KP_AMI_WINDOWS2022:
      return {false, true, true, false, true, 50};  // /dev/sda1: 50Gi
    default:
      return {true, true, true, true, false, 20};  // AL2023 / AL2 /dev/xvda DefaultEBS; Custom: none -> DefaultEBS
  }
}
typedef struct kpo_overhead {
  kp_resource_list kube_reserved, system_reserved, eviction_threshold;
} kpo_overhead;

// ephemeralStorage(info, amiFamily, blockDeviceMappings, instanceStorePolicy) (R:types.go:349-385), in bytes, following
// its control flow: RAID0 with InstanceStorageInfo.TotalSizeInGB -> "%dG"; BDMs: lo.Find(RootVolume) with a volumeSize;
// Custom: the last BDM's volumeSize or DefaultEBS; other families: lo.Find(deviceName == EphemeralBlockDevice()) with a
// volumeSize; then lo.Find(DefaultBlockDeviceMappings(), EphemeralBlockDevice()) -> its volumeSize; DefaultEBS.
struct BDM {
  std::string device;  // "" = nil
  bool has_device;
  bool root;
  bool has_size;
  int64_t size;
};
static int64_t EphemeralStorageBytes(const kp_ec2_info* info, const kp_nodeclass* nc) {
  const int64_t DefaultEBSVolumeSize = 20ll * 1073741824ll;  // R:pkg/providers/amifamily/resolver.go DefaultEBS
  const int fam = nc ? nc->ami_family : KP_AMI_AL2023;
  if (nc && nc->instance_store_policy == KP_INSTANCE_STORE_RAID0) {
    int64_t totalGB = info->instance_storage_gb ? info->instance_storage_gb : info->local_nvme_gb;
    if (totalGB > 0) return totalGB * 1000 * 1000 * 1000;
  }
  std::vector<BDM> bdms;
  for (uint32_t i = 0; nc && nc->block_device_mappings && i < nc->n_block_device_mappings; i++) {
    const kp_block_device_mapping& b = nc->block_device_mappings[i];
    bdms.push_back({b.device_name ? b.device_name : "", b.device_name != nullptr, b.root_volume != 0, b.volume_size >= 0,
                    b.volume_size});
  }
  // EphemeralBlockDevice() and DefaultBlockDeviceMappings() per family (nil device: Custom)
  std::string ephDevice;
  bool hasEphDevice = true;
  std::vector<BDM> defaults;
  switch (fam) {
    case KP_AMI_BOTTLEROCKET:
      ephDevice = "/dev/xvdb";
      defaults = {{"/dev/xvda", true, false, true, 4ll * 1073741824ll}, {"/dev/xvdb", true, false, true, DefaultEBSVolumeSize}};
      break;
    case KP_AMI_WINDOWS2019:
    case KP_AMI_WINDOWS2022:
      ephDevice = "/dev/sda1";
      defaults = {{"/dev/sda1", true, false, true, 50ll * 1073741824ll}};
      break;
    case KP_AMI_CUSTOM:
      hasEphDevice = false;
      break;
    default:
      ephDevice = "/dev/xvda";
      defaults = {{"/dev/xvda", true, false, true, DefaultEBSVolumeSize}};
  }
  if (!bdms.empty()) {
    auto root = std::find_if(bdms.begin(), bdms.end(), [](const BDM& b) { return b.root; });
    if (root != bdms.end() && root->has_size) return root->size;
    if (!hasEphDevice) return bdms.back().has_size ? bdms.back().size : DefaultEBSVolumeSize;
    auto dev = std::find_if(bdms.begin(), bdms.end(), [&](const BDM& b) { return b.has_device && b.device == ephDevice; });
    if (dev != bdms.end() && dev->has_size) return dev->size;
  }
  if (hasEphDevice) {
    auto def = std::find_if(defaults.begin(), defaults.end(), [&](const BDM& b) { return b.device == ephDevice; });
    if (def != defaults.end()) return def->size;
  }
  return DefaultEBSVolumeSize;
}

static int64_t Mi(int64_t x) { return x * 1048576ll * 1000ll; }

static int64_t ENILimitedPods(const kp_ec2_info* info, int reservedENIs) {
  int64_t usable = std::max<int64_t>((int64_t)info->max_enis - reservedENIs, 0);
  if (usable == 0) return 0;
  return usable * ((int64_t)info->ipv4_per_eni - 1) + 2;
}

int32_t kpo_instance_type_resolve(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc,
                                  kp_resource_list* capacity, kpo_overhead* overhead) {
  ResourceList cap;
  cap[KP_RES_CPU] = (int64_t)info->vcpu * 1000;
  // memory(): arm64 loses 64 MiB of CMA; then subtract ceil(bytes*VMMemoryOverheadPercent/1024/1024) MiB
  int64_t mib = info->memory_mib;
  if (info->arch && std::string(info->arch) == "arm64") mib -= 64;
  double bytes = (double)(mib * 1048576ll);
  int64_t ovMiB = (int64_t)std::ceil(bytes * opts->vm_memory_overhead_percent / 1024 / 1024);
  cap[KP_RES_MEMORY] = Mi(mib - ovMiB);
  const AMIFamilyFlags fam = FamilyOf(nc);
  int64_t storageBytes = EphemeralStorageBytes(info, nc);
  cap[KP_RES_EPHEMERAL_STORAGE] = storageBytes * 1000;
  // pods(): maxPods, else ENI-limited (SupportsENILimitedPodDensity), else 110; then podsPerCore (PodsPerCoreEnabled)
  int64_t pods;
  if (nc && nc->max_pods >= 0) pods = nc->max_pods;
  else if (fam.SupportsENILimitedPodDensity) pods = ENILimitedPods(info, opts->reserved_enis);
  else pods = 110;
  if (nc && nc->pods_per_core > 0 && fam.PodsPerCoreEnabled)
    pods = std::min<int64_t>((int64_t)nc->pods_per_core * info->vcpu, pods);
  cap[KP_RES_PODS] = pods * 1000;
  cap[KP_RES_POD_ENI] = (info->in_limits_table && info->trunking) ? (int64_t)info->branch_enis * 1000 : 0;
  std::string gm = info->gpu_manufacturer ? info->gpu_manufacturer : "";
  cap[KP_RES_NVIDIA_GPU] = (gm == "nvidia" ? info->gpu_count : 0) * 1000ll;
  cap[KP_RES_AMD_GPU] = (gm == "amd" ? info->gpu_count : 0) * 1000ll;
  cap[KP_RES_NEURON] = (int64_t)info->neuron_devices * 1000;
  cap[KP_RES_NEURONCORE] = (int64_t)info->neuron_devices * info->neuron_cores_per_device * 1000;
  cap[KP_RES_GAUDI] = (gm == "habana" ? info->gpu_count : 0) * 1000ll;
  cap[KP_RES_EFA] = (int64_t)info->efa * 1000;
  // R:types.go:151-153: types compatible with os In {windows} (getOS: Windows families, amd64) get PrivateIPv4Address
  // = the VPC limits table's IPv4 addresses per interface - 1, 0 when the table lacks the type (:477-484)
  if (fam.Windows && info->arch && std::string(info->arch) == "amd64")
    cap[KP_RES_PRIVATE_IPV4] = info->in_limits_table ? ((int64_t)info->ipv4_per_eni - 1) * 1000 : 0;
  *capacity = ToABI(cap);

  // kubeReservedResources: memory from ENILimitedPods(ctx, info, 0) when UsesENILimitedMemoryOverhead, else pods()
  ResourceList kube;
  kube[KP_RES_MEMORY] = Mi(11 * (fam.UsesENILimitedMemoryOverhead ? ENILimitedPods(info, 0) : pods) + 255);
  kube[KP_RES_EPHEMERAL_STORAGE] = 1073741824ll * 1000;
  struct R {
    int64_t start, end;
    double pct;
  } ranges[4] = {{0, 1000, 0.06}, {1000, 2000, 0.01}, {2000, 4000, 0.005}, {4000, 1ll << 31, 0.0025}};
  int64_t cpuM = cap[KP_RES_CPU];
  for (auto& rg : ranges) {
    if (cpuM >= rg.start) {
      double r = (double)(rg.end - rg.start);
      if (cpuM < rg.end) r = (double)(cpuM - rg.start);
      kube[KP_RES_CPU] = Get(kube, KP_RES_CPU) + (int64_t)(r * rg.pct);
    }
  }
  const kp_kubelet* kl = nc ? nc->kubelet : nullptr;
  ResourceList sys;
  if (kl) {  // lo.Assign(computed, kubeReserved); systemReserved is the map as given
    ResourceList kr = FromABI(kl->kube_reserved), sr = FromABI(kl->system_reserved);
    for (auto& kv : kr) kube[kv.first] = kv.second;
    sys = sr;
  }
  // evictionThreshold: memory 100Mi, ephemeral ceil(storage/100*10); signal maps (evictionHard, then evictionSoft —
  // EvictionSoftEnabled for AL2023) each give a temp list, MaxResources'd together, then assigned over the defaults
  ResourceList ev;
  ev[KP_RES_MEMORY] = Mi(100);
  ev[KP_RES_EPHEMERAL_STORAGE] = (int64_t)std::ceil((double)storageBytes / 100 * 10) * 1000;
  if (kl) {
    auto signal = [](double capacityUnits, const kp_eviction_value& v) -> int64_t {  // computeEvictionSignal
      if (!v.is_percent) return v.milli;
      double p = v.percent;
      if (p == 100) p = 0;  // mustParsePercentage: 100% disables the threshold
      return (int64_t)std::ceil(capacityUnits / 100 * p) * 1000;
    };
    const double memUnits = (double)(mib - ovMiB) * 1048576.0, fsUnits = (double)storageBytes;
    std::vector<std::pair<const kp_eviction_value*, const kp_eviction_value*>> maps;
    if (kl->has_eviction_hard) maps.push_back({&kl->hard_memory_available, &kl->hard_nodefs_available});
    if (kl->has_eviction_soft && fam.EvictionSoftEnabled) maps.push_back({&kl->soft_memory_available, &kl->soft_nodefs_available});
    ResourceList override_;
    for (auto& m : maps) {
      ResourceList temp;
      if (m.first->set) temp[KP_RES_MEMORY] = signal(memUnits, *m.first);
      if (m.second->set) temp[KP_RES_EPHEMERAL_STORAGE] = signal(fsUnits, *m.second);
      for (auto& kv : temp)  // resources.MaxResources
        if (!override_.count(kv.first) || kv.second > override_[kv.first]) override_[kv.first] = kv.second;
    }
    for (auto& kv : override_) ev[kv.first] = kv.second;
  }
  overhead->kube_reserved = ToABI(kube);
  overhead->system_reserved = ToABI(sys);
  overhead->eviction_threshold = ToABI(ev);
  return KP_OK;
}

}  // extern "C"
