// kp_host.cpp — host side of the C ABI (include/kp/kp_abi.h).
//
// Compiles the string-keyed reference objects (InstanceType, NodePool, Pod, Node) into the device data
// model of kp_model.h, owns device memory and the HIP stream, launches the kernels of kp_kernels.hip and
// copies results back. There is no CPU fallback: without a HIP device every compute entry point returns
// KP_E_DEVICE (the Go shim's own CPU path is the fallback).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <arpa/inet.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kp/kp_abi.h"
#include "kp_device.h"
#include "kp_model.h"

using std::map;
using std::string;
using std::vector;

namespace {

thread_local string g_err;
std::atomic<bool> g_host_timing{false};  // kp_overrides.host_timing of the last context that set it (stderr only)
int32_t fail(int32_t code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(KP_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_));   \
  } while (0)

const char* kHostname = "kubernetes.io/hostname";
const char* kZone = "topology.kubernetes.io/zone";
const char* kCapType = "karpenter.sh/capacity-type";
const char* kZoneID = "topology.k8s.aws/zone-id";
const char* kResID = "karpenter.k8s.aws/capacity-reservation-id";
const char* kResType = "karpenter.k8s.aws/capacity-reservation-type";
const char* kNodePool = "karpenter.sh/nodepool";

// karpv1.WellKnownLabels + R:pkg/apis/v1/labels.go:31-56
const std::set<string>& WellKnown() {
  static const std::set<string> s = {
      "karpenter.sh/nodepool", "topology.kubernetes.io/zone", "topology.kubernetes.io/region",
      "node.kubernetes.io/instance-type", "kubernetes.io/arch", "kubernetes.io/os", "karpenter.sh/capacity-type",
      "node.kubernetes.io/windows-build", "karpenter.k8s.aws/capacity-reservation-id",
      "karpenter.k8s.aws/capacity-reservation-type", "karpenter.k8s.aws/instance-hypervisor",
      "karpenter.k8s.aws/instance-encryption-in-transit-supported", "karpenter.k8s.aws/instance-category",
      "karpenter.k8s.aws/instance-family", "karpenter.k8s.aws/instance-generation", "karpenter.k8s.aws/instance-size",
      "karpenter.k8s.aws/instance-local-nvme", "karpenter.k8s.aws/instance-cpu",
      "karpenter.k8s.aws/instance-cpu-manufacturer", "karpenter.k8s.aws/instance-cpu-sustained-clock-speed-mhz",
      "karpenter.k8s.aws/instance-memory", "karpenter.k8s.aws/instance-ebs-bandwidth",
      "karpenter.k8s.aws/instance-network-bandwidth", "karpenter.k8s.aws/instance-gpu-name",
      "karpenter.k8s.aws/instance-gpu-manufacturer", "karpenter.k8s.aws/instance-gpu-count",
      "karpenter.k8s.aws/instance-gpu-memory", "karpenter.k8s.aws/instance-accelerator-name",
      "karpenter.k8s.aws/instance-accelerator-manufacturer", "karpenter.k8s.aws/instance-accelerator-count",
      "topology.k8s.aws/zone-id"};
  return s;
}
string Normalize(const string& k) {  // karpv1.NormalizedLabels (+ R:kwok/operator/operator.go:73)
  static const map<string, string> m = {
      {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
      {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
      {"beta.kubernetes.io/os", "kubernetes.io/os"},
      {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
      {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
      {"topology.ebs.csi.aws.com/zone", "topology.kubernetes.io/zone"},
  };
  auto it = m.find(k);
  return it == m.end() ? k : it->second;
}
bool Atoi(const string& s, int64_t* out) {  // Go strconv.Atoi
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    if (s.size() == 1) return false;
    i = 1;
  }
  unsigned __int128 v = 0;
  const unsigned __int128 lim = (unsigned __int128)std::numeric_limits<int64_t>::max() + (neg ? 1 : 0);
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (unsigned)(s[i] - '0');
    if (v > lim) return false;
  }
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// ------------------------------------------------------------------------------------------------
// raw (string) model
// ------------------------------------------------------------------------------------------------
struct RawReq {
  string key;
  int op;
  vector<string> values;
  int minv;  // < 0 nil
};
using RawReqs = vector<RawReq>;

RawReqs ParseReqs(const kp_requirements& in) {
  RawReqs out;
  for (uint32_t i = 0; i < in.n; i++) {
    const kp_requirement& q = in.items[i];
    RawReq r;
    r.key = Normalize(q.key ? q.key : "");
    r.op = q.op;
    r.minv = q.min_values;
    for (uint32_t j = 0; j < q.n_values; j++) r.values.push_back(q.values[j] ? q.values[j] : "");
    out.push_back(std::move(r));
  }
  return out;
}
RawReqs LabelReqs(const kp_label* l, uint32_t n, bool drop_hostname) {
  RawReqs out;
  out.reserve(n + 1);
  for (uint32_t i = 0; i < n; i++) {
    string k = Normalize(l[i].key ? l[i].key : "");
    if (drop_hostname && k == kHostname) continue;
    out.push_back({k, KP_OP_IN, {l[i].value ? l[i].value : ""}, -1});
  }
  return out;
}

// scheduling.GetHostPorts entries in a canonical form: (protocol, port) group + 16-byte IP (IPv4 as ::ffff:a.b.c.d,
// the form net.ParseIP returns, so IP.Equal of a v4 and its v4-in-v6 spelling holds). Entries with hostPort 0 are
// skipped, as GetHostPorts skips them; an unparsable IP is KP_E_INVAL (the API server validates hostIP).
struct HostPortKey {
  int proto, port;
  std::array<uint8_t, 16> ip;
  bool unspec;
};
bool ParseHostPorts(const kp_host_port* hp, uint32_t n, vector<HostPortKey>* out, string* err) {
  for (uint32_t i = 0; i < n; i++) {
    if (hp[i].port == 0) continue;
    if (hp[i].port < 0 || hp[i].port > 65535 || hp[i].protocol < KP_PROTO_TCP || hp[i].protocol > KP_PROTO_SCTP) {
      *err = "host port " + std::to_string(hp[i].port) + "/" + std::to_string(hp[i].protocol);
      return false;
    }
    HostPortKey k;
    k.proto = hp[i].protocol;
    k.port = hp[i].port;
    k.ip.fill(0);
    const string ip = hp[i].ip && hp[i].ip[0] ? hp[i].ip : "0.0.0.0";
    uint8_t v4[4];
    if (inet_pton(AF_INET, ip.c_str(), v4) == 1) {
      k.ip[10] = k.ip[11] = 0xFF;
      memcpy(&k.ip[12], v4, 4);
    } else if (inet_pton(AF_INET6, ip.c_str(), k.ip.data()) != 1) {
      *err = "host IP '" + ip + "'";
      return false;
    }
    static const uint8_t v4z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF, 0, 0, 0, 0};
    static const uint8_t v6z[16] = {0};
    k.unspec = memcmp(k.ip.data(), v4z, 16) == 0 || memcmp(k.ip.data(), v6z, 16) == 0;
    out->push_back(k);
  }
  return true;
}

struct HostOffering {
  string ct, zone, zid;
  bool has_zone, has_zid;
  double price;
  bool available;
  string rid, rt;  // capacity-reservation-id / -type In {..}; DoesNotExist when !has_rid / !has_rt
  bool has_rid = false, has_rt = false;
  int32_t rcap = 0;  // ReservationCapacity
};
struct HostType {
  string name;
  RawReqs reqs;
  int64_t cap[KP_NRES];
  int64_t ovh[KP_NRES];
  uint32_t cap_present;
  vector<HostOffering> offs;
};

}  // namespace

namespace {
struct SolveBase;
}

struct kp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  kp_options opts;
  kp_overrides ov{};  // kp_ctx_set_overrides (tests, measurement); all 0 = production
  std::recursive_mutex mu;  // recursive: the general simulation path runs whole Solves under the cluster plan's lock
  // resident compiled catalogues + templates of recent Solves (most recent last), see SolveBase
  vector<std::shared_ptr<SolveBase>> bases;
  uint64_t base_hits = 0, base_misses = 0;
  // per-Solve device arena handed back by kp_solve_plan_destroy and reused by the next kp_solve_prepare
  void* spare = nullptr;
  size_t spare_bytes = 0;
  // kp_ctx_destroy's reference plus one per live dependent (catalogue, plan, communicator): the context is freed
  // when the last goes, so a dependent may be destroyed after the context (any order, e.g. a garbage collector's)
  std::atomic<int> refs{1};
};
static void CtxFree(kp_ctx* c) {
  (void)hipSetDevice(c->device);
  c->bases.clear();
  if (c->spare) (void)hipFree(c->spare);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev2) (void)hipEventDestroy(c->ev2);
  if (c->ev3) (void)hipEventDestroy(c->ev3);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}
inline void CtxUnref(kp_ctx* c) {
  if (c && c->refs.fetch_sub(1) == 1) CtxFree(c);
}
// A dependent's context pointer holding a reference (assignment takes one, destruction drops it).
struct CtxRef {
  kp_ctx* p = nullptr;
  CtxRef() = default;
  CtxRef(const CtxRef&) = delete;
  CtxRef& operator=(const CtxRef&) = delete;
  CtxRef& operator=(kp_ctx* c) {
    if (c) c->refs.fetch_add(1);
    CtxUnref(p);
    p = c;
    return *this;
  }
  ~CtxRef() { CtxUnref(p); }
  kp_ctx* operator->() const { return p; }
  operator kp_ctx*() const { return p; }
};

struct kp_catalog {
  CtxRef ctx;
  uint64_t seqnum;
  uint64_t uid;  // process-unique identity (a new upload never reuses one, unlike its address)
  vector<HostType> types;
  bool reservations = false;  // some offering carries a capacity-reservation id or type
  // false once kp_catalog_destroy ran: plans and cached bases that compiled this catalogue hold the token and refuse
  // to run (or refresh) instead of reading a freed catalogue
  std::shared_ptr<bool> alive = std::make_shared<bool>(true);
};

namespace {

// ------------------------------------------------------------------------------------------------
// dictionary
// ------------------------------------------------------------------------------------------------
struct Dict {
  vector<string> keys;
  std::unordered_map<string, int> key_id;
  vector<vector<string>> vals;
  vector<std::unordered_map<string, int>> val_id;  // value -> bit (global)
  DevDict dd;
  vector<int64_t> vint;  // [W*64]
  int key(const string& k) const {
    auto it = key_id.find(k);
    return it == key_id.end() ? -1 : it->second;
  }
  int bit(int k, const string& v) const {
    auto it = val_id[k].find(v);
    return it == val_id[k].end() ? -1 : it->second;
  }
};

struct DictBuilder {
  map<string, bool> bounded;  // key -> needs bound slot
  map<string, std::set<string>> values;
  void addReqs(const RawReqs& rs) {
    for (auto& r : rs) {
      auto& b = bounded[r.key];
      if (r.op == KP_OP_GT || r.op == KP_OP_LT || r.minv >= 0) b = true;
      auto& s = values[r.key];
      if (r.op == KP_OP_IN || r.op == KP_OP_NOT_IN) s.insert(r.values.begin(), r.values.end());
    }
  }
  void addLabel(const string& k, const string& v) {
    bounded[k];
    values[k].insert(v);
  }
  int32_t build(Dict& d) {
    vector<string> order;
    for (auto& kv : bounded)
      if (kv.second) order.push_back(kv.first);
    const int KB = (int)order.size();
    if (KB > KP_MAX_BOUND_KEYS) return fail(KP_E_UNSUPPORTED, "%d keys with Gt/Lt/minValues (max %d)", KB, KP_MAX_BOUND_KEYS);
    for (auto& kv : bounded)
      if (!kv.second) order.push_back(kv.first);
    if ((int)order.size() > KP_MAX_KEYS) return fail(KP_E_UNSUPPORTED, "%zu label keys (max %d)", order.size(), KP_MAX_KEYS);
    memset(&d.dd, 0, sizeof(d.dd));
    d.keys = order;
    d.vals.assign(order.size(), {});
    d.val_id.assign(order.size(), {});
    const int K = (int)order.size();
    int w = K;  // words 0..K-1 are the keys' first words; overflow words follow
    for (int k = 0; k < K; k++) {
      d.key_id[order[k]] = k;
      auto& s = values[order[k]];
      d.vals[k].assign(s.begin(), s.end());
      const int nw = std::max<int>(1, (int)((s.size() + 63) / 64));
      d.dd.wofs[k] = k;
      d.dd.ovf[k] = nw > 1 ? w : -1;
      d.dd.nval[k] = (int)s.size();
      d.dd.wkey[k] = (int8_t)k;
      if (nw > 1) {
        if (w + nw - 1 > KP_MAX_WORDS) return fail(KP_E_UNSUPPORTED, "label values need > %d words", KP_MAX_WORDS);
        d.dd.multiword |= 1ull << k;
        for (int i = 0; i < nw - 1; i++) {
          d.dd.wkey[w + i] = (int8_t)k;
          d.dd.ovfmask[k] |= 1ull << (w + i);
        }
        w += nw - 1;
      }
      int b = 0;
      for (auto& v : d.vals[k]) {
        const int word = b < 64 ? k : d.dd.ovf[k] + b / 64 - 1;
        d.val_id[k][v] = word * 64 + b % 64;
        d.dd.validbits[word] |= 1ull << (b % 64);
        b++;
      }
    }
    d.dd.firstmask = K >= 64 ? ~0ull : ((1ull << K) - 1);
    for (int i = w; i < KP_MAX_WORDS; i++) d.dd.wkey[i] = -1;
    d.dd.K = (int)order.size();
    d.dd.W = w;
    d.dd.KB = KB;
    d.vint.assign((size_t)std::max(w, 1) * 64, 0);
    for (size_t k = 0; k < order.size(); k++)
      for (auto& kv : d.val_id[k]) {
        int64_t x;
        if (Atoi(kv.first, &x)) {
          d.vint[kv.second] = x;
          d.dd.vint_ok[kv.second / 64] |= 1ull << (kv.second % 64);
        }
      }
    for (size_t k = 0; k < order.size(); k++)
      if (WellKnown().count(order[k])) d.dd.wellknown |= 1ull << k;
    int rk = d.key(kResID), tk = d.key(kResType);
    d.dd.resid_key_bit = rk >= 0 ? 1ull << rk : 0;
    d.dd.restype_key_bit = tk >= 0 ? 1ull << tk : 0;
    d.dd.offer_keys = d.dd.resid_key_bit | d.dd.restype_key_bit;
    for (const char* k : {kCapType, kZone, kZoneID})
      if (d.key(k) >= 0) d.dd.offer_keys |= 1ull << d.key(k);
    return KP_OK;
  }
};

// ------------------------------------------------------------------------------------------------
// host requirement algebra on KReqs (same encoding the device uses)
// ------------------------------------------------------------------------------------------------
bool Within(const Dict& d, int bit, bool hg, int64_t gt, bool hl, int64_t lt) {
  if (!hg && !hl) return true;
  if (!((d.dd.vint_ok[bit / 64] >> (bit % 64)) & 1)) return false;
  int64_t x = d.vint[bit];
  if (hg && gt >= x) return false;
  if (hl && lt <= x) return false;
  return true;
}
int nwords(const Dict& d, int k) { return std::max(1, (d.dd.nval[k] + 63) / 64); }
int kw(const Dict& d, int k, int i) { return i == 0 ? k : d.dd.ovf[k] + i - 1; }  // i-th word of key k

KReqs Single(const Dict& d, const RawReq& r) {
  KReqs q;
  memset(&q, 0, sizeof q);
  const int k = d.key(r.key);
  q.present = 1ull << k;
  if (r.minv >= 0) {
    q.hmin = 1ull << k;
    q.minv[k] = r.minv;
  }
  auto setvals = [&]() {
    for (auto& v : r.values) {
      int b = d.bit(k, v);
      q.vals[b / 64] |= 1ull << (b % 64);
    }
  };
  switch (r.op) {
    case KP_OP_IN:
      setvals();
      break;
    case KP_OP_NOT_IN:
      q.compl_ = 1ull << k;
      setvals();
      break;
    case KP_OP_EXISTS:
      q.compl_ = 1ull << k;
      break;
    case KP_OP_DOES_NOT_EXIST:
      break;
    case KP_OP_GT:
    case KP_OP_LT: {
      q.compl_ = 1ull << k;
      int64_t x = 0;
      Atoi(r.values.empty() ? string() : r.values[0], &x);
      if (r.op == KP_OP_GT) {
        q.hgt = 1ull << k;
        q.gt[k] = x;
      } else {
        q.hlt = 1ull << k;
        q.lt[k] = x;
      }
      break;
    }
  }
  return q;
}

// A = A.Add(B) per key (Requirement.Intersection for shared keys).
void HostAdd(const Dict& d, KReqs& A, const KReqs& B) {
  // B's keys in increasing order (each key is independent of the others)
  for (uint64_t km = B.present & (d.dd.K >= 64 ? ~0ull : (1ull << d.dd.K) - 1); km; km &= km - 1) {
    const int k = __builtin_ctzll(km);
    const uint64_t kb = 1ull << k;
    const int nw = nwords(d, k);
    const bool bnd = k < KP_MAX_BOUND_KEYS;
    if (!(A.present & kb)) {
      A.present |= kb;
      A.compl_ = (A.compl_ & ~kb) | (B.compl_ & kb);
      A.hgt = (A.hgt & ~kb) | (B.hgt & kb);
      A.hlt = (A.hlt & ~kb) | (B.hlt & kb);
      A.hmin = (A.hmin & ~kb) | (B.hmin & kb);
      if (bnd) {
        A.gt[k] = B.gt[k];
        A.lt[k] = B.lt[k];
        A.minv[k] = B.minv[k];
      }
      for (int i = 0; i < nw; i++) A.vals[kw(d, k, i)] = B.vals[kw(d, k, i)];
      continue;
    }
    const bool c1 = A.compl_ & kb, c2 = B.compl_ & kb;
    const bool ag = A.hgt & kb, bg = B.hgt & kb, al = A.hlt & kb, bl = B.hlt & kb;
    const bool hg = ag || bg, hl = al || bl;
    int64_t gt = 0, lt = 0;
    if (bnd) {
      gt = ag && bg ? std::max(A.gt[k], B.gt[k]) : (ag ? A.gt[k] : B.gt[k]);
      lt = al && bl ? std::min(A.lt[k], B.lt[k]) : (al ? A.lt[k] : B.lt[k]);
      const bool am = A.hmin & kb, bm = B.hmin & kb;
      A.minv[k] = am && bm ? std::max(A.minv[k], B.minv[k]) : (am ? A.minv[k] : B.minv[k]);
    }
    A.hmin |= B.hmin & kb;
    if (hg && hl && gt >= lt) {  // DoesNotExist
      A.compl_ &= ~kb;
      A.hgt &= ~kb;
      A.hlt &= ~kb;
      for (int i = 0; i < nw; i++) A.vals[kw(d, k, i)] = 0;
      continue;
    }
    for (int i = 0; i < nw; i++) {
      const int w = kw(d, k, i);
      const uint64_t a = A.vals[w], b = B.vals[w];
      uint64_t v = (c1 && c2) ? (a | b) : c1 ? (b & ~a) : c2 ? (a & ~b) : (a & b);
      if (hg || hl) {
        uint64_t m = v, o = 0;
        while (m) {
          int bb = __builtin_ctzll(m);
          m &= m - 1;
          if (Within(d, w * 64 + bb, hg, gt, hl, lt)) o |= 1ull << bb;
        }
        v = o;
      }
      A.vals[w] = v;
    }
    const bool c = c1 && c2;
    if (c) {
      A.compl_ |= kb;
      if (hg) A.hgt |= kb, A.gt[k] = gt;
      if (hl) A.hlt |= kb, A.lt[k] = lt;
    } else {
      A.compl_ &= ~kb;
      A.hgt &= ~kb;
      A.hlt &= ~kb;
    }
  }
}

KReqs Compile(const Dict& d, const RawReqs& rs) {
  KReqs q;
  memset(&q, 0, sizeof q);
  for (auto& r : rs) HostAdd(d, q, Single(d, r));
  return q;
}
bool KeyNonEmptyVals(const Dict& d, const KReqs& q, int k) {
  for (int i = 0; i < nwords(d, k); i++)
    if (q.vals[kw(d, k, i)]) return true;
  return false;
}
uint64_t NegOp(const Dict& d, const KReqs& q) {
  uint64_t m = 0;
  for (int k = 0; k < d.dd.K; k++) {
    if (!((q.present >> k) & 1)) continue;
    bool c = (q.compl_ >> k) & 1, nz = KeyNonEmptyVals(d, q, k);
    if ((c && nz) || (!c && !nz)) m |= 1ull << k;
  }
  return m;
}
bool Has(const Dict& d, const KReqs& q, int k, int bit) {
  if (!((q.present >> k) & 1)) return true;
  bool in = (q.vals[bit / 64] >> (bit % 64)) & 1;
  if ((q.compl_ >> k) & 1) {
    const bool bnd = k < KP_MAX_BOUND_KEYS;
    return !in && Within(d, bit, bnd && ((q.hgt >> k) & 1), bnd ? q.gt[k] : 0, bnd && ((q.hlt >> k) & 1),
                         bnd ? q.lt[k] : 0);
  }
  return in;
}

// ------------------------------------------------------------------------------------------------
// catalogue compile (per solve dictionary)
// ------------------------------------------------------------------------------------------------
struct HostCat {
  int T = 0, S = 0;
  vector<KReqs> treqs;
  vector<uint64_t> TM, DNE, NOKEY;    // [nbits][TW], [K][TW], [K][TW]
  vector<int64_t> alloc, cap;         // [R][T]
  vector<uint64_t> nonneg;            // [TW]
  vector<int64_t> fit_vals;           // [R][T]
  vector<int32_t> fit_n;              // [R]
  vector<uint64_t> fit_mask;          // [R][T][TW]
  vector<uint64_t> offer_avail;       // [C][TW]
  vector<double> price;               // [T][C]
  vector<double> price_cm;            // [C][S]
  vector<double> price_sub;           // [2^C][S] (C <= KP_SUB_MAX_C)
  vector<uint32_t> name_rank;         // [T]
  vector<uint16_t> code;              // [K][T]
  vector<uint64_t> multi;             // [K][T]
  vector<uint64_t> custom_nonneg;     // [T]
  uint64_t multi_valued = 0;
  uint64_t custom_any = 0;            // OR of custom_nonneg
};

struct ClassKey {
  int ct, zone, zid, rid = -1, rt = -1;
  bool operator<(const ClassKey& o) const {
    return std::tie(ct, zone, zid, rid, rt) < std::tie(o.ct, o.zone, o.zid, o.rid, o.rt);
  }
};
// An offering's class: its label values as dictionary bits (-1: no such requirement / DoesNotExist).
ClassKey ClassOf(const Dict& d, const HostOffering& o) {
  return {d.bit(d.key(kCapType), o.ct), o.has_zone ? d.bit(d.key(kZone), o.zone) : -1,
          o.has_zid ? d.bit(d.key(kZoneID), o.zid) : -1, o.has_rid ? d.bit(d.key(kResID), o.rid) : -1,
          o.has_rt ? d.bit(d.key(kResType), o.rt) : -1};
}
OfferClass ClassOfKey(const ClassKey& k) {
  return {(int16_t)k.ct, (int16_t)k.zone, (int16_t)k.zid, (int16_t)k.rid, (int16_t)k.rt, {0, 0, 0}};
}
ClassKey KeyOfClass(const OfferClass& c) { return {c.ct_bit, c.zone_bit, c.zid_bit, c.rid_bit, c.rt_bit}; }

// Offering section of a compiled catalogue: available classes per type, cheapest price per (type, class), and the
// class-major copy (offering.go:115-147 createOfferings: Available = !ICE && hasPrice && zone offered). Also the
// whole of an ICE refresh (kp_filter_refresh): availability and price are the only inputs an ICE mark changes.
void FillOfferings(const Dict& d, const vector<HostType>& types, int TW, const map<ClassKey, int>& classes,
                   HostCat& hc) {
  const int T = hc.T, S = hc.S;
  const int C = (int)classes.size();
  hc.offer_avail.assign((size_t)C * TW, 0);
  hc.price.assign((size_t)T * C, std::numeric_limits<double>::infinity());
  for (int t = 0; t < T; t++)
    for (auto& o : types[t].offs) {
      const int c = classes.at(ClassOf(d, o));
      if (!o.available) continue;
      hc.offer_avail[(size_t)c * TW + t / 64] |= 1ull << (t % 64);
      double& p = hc.price[(size_t)t * C + c];
      if (o.price < p) p = o.price;
    }
  hc.price_cm.assign((size_t)C * S, std::numeric_limits<double>::infinity());  // row stride S (= D.T)
  for (int t = 0; t < T; t++)
    for (int c = 0; c < C; c++) hc.price_cm[(size_t)c * S + t] = hc.price[(size_t)t * C + c];
  // cheapest over a row's compatible class set in one gather: min over each subset m, built from m & (m - 1)
  hc.price_sub.clear();
  if (C <= KP_SUB_MAX_C) {
    hc.price_sub.assign((size_t)S << C, std::numeric_limits<double>::infinity());
    for (size_t m = 1; m < ((size_t)1 << C); m++) {
      const int c = __builtin_ctzll(m);
      const double* prev = &hc.price_sub[(m & (m - 1)) * S];
      double* cur = &hc.price_sub[m * S];
      for (int t = 0; t < T; t++) cur[t] = std::min(prev[t], hc.price[(size_t)t * C + c]);
    }
  }
}

int32_t CompileCatalog(const Dict& d, const vector<HostType>& types, int TW, map<ClassKey, int>& classes, HostCat& hc) {
  const int T = (int)types.size(), K = d.dd.K, NB = d.dd.W * 64;
  const int S = std::max(d.dd.T, T);  // row stride shared by every catalogue of the solve (device uses D.T)
  hc.T = T;
  hc.S = S;
  hc.treqs.resize(T);
  hc.TM.assign((size_t)NB * TW, 0);
  hc.DNE.assign((size_t)K * TW, 0);
  hc.NOKEY.assign((size_t)K * TW, 0);
  hc.code.assign((size_t)K * S, 0xFFFF);
  hc.multi.assign((size_t)K * S, 0);
  hc.custom_nonneg.assign(S, 0);
  for (int t = 0; t < T; t++) {
    KReqs q = Compile(d, types[t].reqs);
    hc.treqs[t] = q;
    const uint64_t tb = 1ull << (t % 64);
    const int tw = t / 64;
    const uint64_t neg = NegOp(d, q);
    for (int k = 0; k < K; k++) {
      const uint64_t kb = 1ull << k;
      if (!(q.present & kb)) {
        hc.NOKEY[(size_t)k * TW + tw] |= tb;
        continue;
      }
      if ((q.compl_ & kb) || (q.hgt & kb) || (q.hlt & kb))
        return fail(KP_E_UNSUPPORTED, "instance type %s: requirement %s is not In/DoesNotExist", types[t].name.c_str(),
                    d.keys[k].c_str());
      if (!(d.dd.wellknown & kb) && !(neg & kb)) {
        hc.custom_nonneg[t] |= kb;
        hc.custom_any |= kb;
      }
      int cnt = 0, last = -1;
      for (int wi = 0, w = kw(d, k, 0); wi < nwords(d, k); wi++, w = wi < nwords(d, k) ? kw(d, k, wi) : 0) {
        uint64_t m = q.vals[w];
        while (m) {
          int b = __builtin_ctzll(m);
          m &= m - 1;
          int bit = w * 64 + b;
          hc.TM[(size_t)bit * TW + tw] |= tb;
          cnt++;
          last = bit;
        }
      }
      if (cnt == 0) {
        hc.DNE[(size_t)k * TW + tw] |= tb;
        hc.code[(size_t)k * S + t] = 0xFFFE;
      } else if (cnt == 1) {
        hc.code[(size_t)k * S + t] = (uint16_t)last;
      } else {
        if (d.dd.nval[k] > 64) return fail(KP_E_UNSUPPORTED, "multi-valued key %s has > 64 values", d.keys[k].c_str());
        hc.multi_valued |= kb;
        hc.code[(size_t)k * S + t] = 0xFFFD;
        hc.multi[(size_t)k * S + t] = q.vals[d.dd.wofs[k]];
      }
    }
  }
  for (int k = 0; k < K; k++)  // keys whose types are multi-valued keep multi masks for every type
    if ((hc.multi_valued >> k) & 1)
      for (int t = 0; t < T; t++) {
        uint16_t& c = hc.code[(size_t)k * S + t];
        if (c < 0xFFFD) {
          hc.multi[(size_t)k * S + t] = 1ull << (c % 64);
          c = 0xFFFD;
        }
      }
  // resources
  hc.alloc.assign((size_t)KP_NRES * S, 0);
  hc.cap.assign((size_t)KP_NRES * S, 0);
  hc.nonneg.assign(TW, 0);
  for (int t = 0; t < T; t++) {
    bool nn = true;
    for (int r = 0; r < KP_NRES; r++) {
      const bool pr = (types[t].cap_present >> r) & 1;
      const int64_t c = pr ? types[t].cap[r] : 0;
      const int64_t a = pr ? c - types[t].ovh[r] : 0;  // resources.Subtract(capacity, overhead): capacity keys
      hc.cap[(size_t)r * S + t] = c;
      hc.alloc[(size_t)r * S + t] = a;
      if (pr && a < 0) nn = false;
    }
    if (nn) hc.nonneg[t / 64] |= 1ull << (t % 64);
  }
  hc.fit_vals.assign((size_t)KP_NRES * S, 0);
  hc.fit_n.assign(KP_NRES, 0);
  hc.fit_mask.assign((size_t)KP_NRES * S * TW, 0);
  for (int r = 0; r < KP_NRES; r++) {
    vector<int64_t> v(hc.alloc.begin() + (size_t)r * S, hc.alloc.begin() + (size_t)r * S + T);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    hc.fit_n[r] = (int)v.size();
    std::copy(v.begin(), v.end(), hc.fit_vals.begin() + (size_t)r * S);
    // fit_mask[r][j] = types with alloc >= v[j]: build from the top down
    vector<uint64_t> acc(TW, 0);
    vector<std::pair<int64_t, int>> byv;
    for (int t = 0; t < T; t++) byv.push_back({hc.alloc[(size_t)r * S + t], t});
    std::sort(byv.begin(), byv.end());
    int p = T - 1;
    for (int j = (int)v.size() - 1; j >= 0; j--) {
      while (p >= 0 && byv[p].first >= v[j]) {
        acc[byv[p].second / 64] |= 1ull << (byv[p].second % 64);
        p--;
      }
      std::copy(acc.begin(), acc.end(), hc.fit_mask.begin() + ((size_t)r * S + j) * TW);
    }
  }
  FillOfferings(d, types, TW, classes, hc);
  vector<int> idx(T);
  for (int t = 0; t < T; t++) idx[t] = t;
  std::sort(idx.begin(), idx.end(), [&](int a, int b) { return types[a].name < types[b].name; });
  hc.name_rank.assign(S, 0);
  for (int i = 0; i < T; i++) hc.name_rank[idx[i]] = (uint32_t)i;
  return KP_OK;
}

// Pass_k(q_k) over the catalogue (host version, every key of q): NOKEY ∪ ∪_{Has(v)} TM[v] ∪ (negop ? DNE)
void HostFilterTypes(const Dict& d, const HostCat& hc, const KReqs& q, int TW, const int64_t* total,
                     vector<uint64_t>& X) {
  const uint64_t neg = NegOp(d, q);
  for (int k = 0; k < d.dd.K; k++) {
    if (!((q.present >> k) & 1)) continue;
    vector<uint64_t> acc(TW, 0);
    for (int w = 0; w < TW; w++) acc[w] = hc.NOKEY[(size_t)k * TW + w] | (((neg >> k) & 1) ? hc.DNE[(size_t)k * TW + w] : 0);
    for (int wi = 0, w = kw(d, k, 0); wi < nwords(d, k); wi++, w = wi < nwords(d, k) ? kw(d, k, wi) : 0) {
      uint64_t m = d.dd.validbits[w];
      while (m) {
        int b = __builtin_ctzll(m);
        m &= m - 1;
        if (Has(d, q, k, w * 64 + b))
          for (int x = 0; x < TW; x++) acc[x] |= hc.TM[(size_t)(w * 64 + b) * TW + x];
      }
    }
    for (int w = 0; w < TW; w++) X[w] &= acc[w];
  }
  // Fits(total, allocatable)
  for (int t = 0; t < hc.T; t++) {
    bool ok = (hc.nonneg[t / 64] >> (t % 64)) & 1;
    for (int r = 0; r < KP_NRES && ok; r++)
      if (total[r] > 0 && total[r] > hc.alloc[(size_t)r * hc.S + t]) ok = false;
    if (!ok) X[t / 64] &= ~(1ull << (t % 64));
  }
}

uint64_t HostAllowedClasses(const Dict& d, const KReqs& q, const vector<OfferClass>& cls) {
  const uint64_t neg = NegOp(d, q);
  // a reservation key the offering does not carry is DoesNotExist: compatible when the query leaves the key out or
  // admits its absence (NotIn / DoesNotExist)
  const bool res_ok = !(q.present & d.dd.resid_key_bit) || (neg & d.dd.resid_key_bit);
  const bool rt_ok = !(q.present & d.dd.restype_key_bit) || (neg & d.dd.restype_key_bit);
  uint64_t m = 0;
  auto keyof = [&](int bit) { return (int)d.dd.wkey[bit / 64]; };
  for (size_t c = 0; c < cls.size(); c++) {
    bool ok = Has(d, q, keyof(cls[c].ct_bit), cls[c].ct_bit);
    if (cls[c].zone_bit >= 0) ok = ok && Has(d, q, keyof(cls[c].zone_bit), cls[c].zone_bit);
    if (cls[c].zid_bit >= 0) ok = ok && Has(d, q, keyof(cls[c].zid_bit), cls[c].zid_bit);
    ok = ok && (cls[c].rid_bit >= 0 ? Has(d, q, keyof(cls[c].rid_bit), cls[c].rid_bit) : res_ok);
    ok = ok && (cls[c].rt_bit >= 0 ? Has(d, q, keyof(cls[c].rt_bit), cls[c].rt_bit) : rt_ok);
    if (ok) m |= 1ull << c;
  }
  return m;
}

int CountDistinct(const Dict& d, const HostCat& hc, int k, const vector<int>& types) {
  std::set<int> vals;
  for (int t : types) {
    const KReqs& q = hc.treqs[t];
    for (int wi = 0, w = kw(d, k, 0); wi < nwords(d, k); wi++, w = wi < nwords(d, k) ? kw(d, k, wi) : 0) {
      uint64_t m = q.vals[w];
      while (m) {
        int b = __builtin_ctzll(m);
        m &= m - 1;
        vals.insert(w * 64 + b);
      }
    }
  }
  return (int)vals.size();
}
bool HostMinValuesOK(const Dict& d, const HostCat& hc, const KReqs& q, const vector<int>& types) {
  for (int k = 0; k < d.dd.K; k++) {
    if (!((q.hmin >> k) & 1) || !((q.present >> k) & 1)) continue;
    if (CountDistinct(d, hc, k, types) < q.minv[k]) return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// device buffer arena: everything of one solve in one allocation
// ------------------------------------------------------------------------------------------------
// Host image of one device allocation: put()/reserve() lay out host-initialised regions (uploaded in one copy),
// reserve_dev() appends device-only regions after them (no host backing, nothing to zero or copy).
struct Blob {
  vector<uint8_t> host;
  size_t dev_end = 0;  // > 0 once device-only regions were appended
  template <class T>
  size_t put(const T* p, size_t n) {
    size_t off = (host.size() + 255) & ~(size_t)255;
    host.resize(off + n * sizeof(T));
    if (n) memcpy(host.data() + off, p, n * sizeof(T));
    return off;
  }
  template <class T>
  size_t put(const vector<T>& v) {
    return put(v.data(), v.size());
  }
  size_t reserve(size_t bytes) {
    size_t off = (host.size() + 255) & ~(size_t)255;
    host.resize(off + bytes);
    return off;
  }
  size_t reserve_dev(size_t bytes) {
    size_t off = (std::max(host.size(), dev_end) + 255) & ~(size_t)255;
    dev_end = off + bytes;
    return off;
  }
  size_t total() const { return std::max(host.size(), dev_end); }
};

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { reset(); }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t bytes) {
    reset();
    hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 1));
    if (e == hipSuccess) n = bytes;
    else p = nullptr;
    return e;
  }
};

}  // namespace

namespace {
// A NodeClaim's final requirements as upstream Requirements.NodeSelectorRequirements() renders them
// (Gt, then Lt, then NotIn/Exists, then In/DoesNotExist), keys in byte order, values sorted. The hostname
// placeholder is not part of the dictionary, as FinalizeScheduling drops it.
struct ReqOut {
  vector<string> keys;
  vector<vector<string>> vals;
  vector<vector<const char*>> ptrs;
  vector<kp_requirement> items;
};
std::shared_ptr<ReqOut> DecodeReqs(const Dict& d, const KReqs& q) {
  auto o = std::make_shared<ReqOut>();
  vector<int> ks;
  for (int k = 0; k < d.dd.K; k++)
    if (((q.present >> k) & 1) && d.keys[k] != kHostname) ks.push_back(k);  // (the NodeClaim's placeholder)
  std::sort(ks.begin(), ks.end(), [&](int a, int b) { return d.keys[a] < d.keys[b]; });
  for (int k : ks) {
    const bool bnd = k < KP_MAX_BOUND_KEYS, c = (q.compl_ >> k) & 1;
    kp_requirement it;
    memset(&it, 0, sizeof it);
    vector<string> v;
    if (c && bnd && ((q.hgt >> k) & 1)) {
      it.op = KP_OP_GT;
      v.push_back(std::to_string(q.gt[k]));
    } else if (c && bnd && ((q.hlt >> k) & 1)) {
      it.op = KP_OP_LT;
      v.push_back(std::to_string(q.lt[k]));
    } else {
      for (int i = 0; i < nwords(d, k); i++) {
        const int w = kw(d, k, i);
        uint64_t m = q.vals[w];
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          v.push_back(d.vals[k][(size_t)i * 64 + b]);  // ordinal = i*64 + b; dictionary values are sorted
        }
      }
      it.op = c ? (v.empty() ? KP_OP_EXISTS : KP_OP_NOT_IN) : (v.empty() ? KP_OP_DOES_NOT_EXIST : KP_OP_IN);
    }
    it.min_values = (bnd && ((q.hmin >> k) & 1)) ? q.minv[k] : -1;
    o->keys.push_back(d.keys[k]);
    o->vals.push_back(std::move(v));
    o->items.push_back(it);
  }
  o->ptrs.resize(o->vals.size());
  for (size_t i = 0; i < o->items.size(); i++) {
    for (auto& x : o->vals[i]) o->ptrs[i].push_back(x.c_str());
    o->items[i].key = o->keys[i].c_str();
    o->items[i].values = o->ptrs[i].data();
    o->items[i].n_values = (uint32_t)o->ptrs[i].size();
  }
  return o;
}
}  // namespace

struct kp_solve_result {
  vector<int32_t> placement;
  struct NC {
    uint32_t nodepool, n_remaining;
    vector<uint32_t> pods, options;
    kp_resource_list requests;
    std::shared_ptr<ReqOut> reqs;
  };
  vector<NC> ncs;
  kp_solve_stats stats;
  vector<KReqs> fin;     // per NodeClaim: final requirements (device encoding), for in-library callers
  vector<int> nc_cat;    // per NodeClaim: catalogue of its template
};

extern "C" {

const char* kp_last_error(void) { return g_err.c_str(); }
int32_t kp_abi_version(void) { return KP_ABI_VERSION; }

int32_t kp_ctx_create(const kp_options* opts, kp_ctx** out) {
  if (!out) return fail(KP_E_INVAL, "out is null");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return fail(KP_E_DEVICE, "no HIP device: %s", hipGetErrorString(e));
  auto* c = new kp_ctx();
  c->opts = opts ? *opts : kp_options{0.075, 0, 0};
  c->device = c->opts.device;
  if (c->device < 0 || c->device >= n) {
    delete c;
    return fail(KP_E_INVAL, "device %d out of range", opts ? opts->device : 0);
  }
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->ev2) != hipSuccess || hipEventCreate(&c->ev3) != hipSuccess) {
    delete c;
    return fail(KP_E_DEVICE, "stream/event creation failed");
  }
  *out = c;
  return KP_OK;
}
void kp_ctx_destroy(kp_ctx* c) { CtxUnref(c); }

int32_t kp_ctx_set_overrides(kp_ctx* ctx, const kp_overrides* ov) {
  if (!ctx) return fail(KP_E_INVAL, "null argument");
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  ctx->ov = ov ? *ov : kp_overrides{};
  g_host_timing.store(ctx->ov.host_timing != 0);
  return KP_OK;
}
int32_t kp_ctx_get_overrides(const kp_ctx* ctx, kp_overrides* out) {
  if (!ctx || !out) return fail(KP_E_INVAL, "null argument");
  *out = ctx->ov;
  return KP_OK;
}


int32_t kp_catalog_upload(kp_ctx* ctx, const kp_catalog_desc* desc, uint64_t seqnum, kp_catalog** out) {
  if (!desc || !out) return fail(KP_E_INVAL, "null argument");  // ctx NULL: host-only (kp_solve_validate)
  if (desc->n_types > 4096) return fail(KP_E_UNSUPPORTED, "%u instance types (max 4096)", desc->n_types);
  static std::atomic<uint64_t> next_uid{1};
  auto* c = new kp_catalog();
  c->ctx = ctx;
  c->seqnum = seqnum;
  c->uid = next_uid.fetch_add(1);
  for (uint32_t i = 0; i < desc->n_types; i++) {
    const kp_instance_type& t = desc->types[i];
    HostType h;
    h.name = t.name ? t.name : "";
    h.reqs = ParseReqs(t.requirements);
    for (int r = 0; r < KP_NRES; r++) {
      h.cap[r] = t.capacity.milli[r];
      h.ovh[r] = (t.overhead.present >> r) & 1 ? t.overhead.milli[r] : 0;
    }
    h.cap_present = t.capacity.present;
    for (uint32_t j = 0; j < t.n_offerings; j++) {
      const kp_offering& o = t.offerings[j];
      h.offs.push_back({o.capacity_type ? o.capacity_type : "", o.zone ? o.zone : "", o.zone_id ? o.zone_id : "",
                        o.zone != nullptr, o.zone_id != nullptr, o.price, o.available != 0});
      HostOffering& ho = h.offs.back();
      ho.has_rid = o.reservation_id != nullptr;
      ho.has_rt = o.reservation_type != nullptr;
      if (ho.has_rid) ho.rid = o.reservation_id;
      if (ho.has_rt) ho.rt = o.reservation_type;
      ho.rcap = o.reservation_capacity;
      c->reservations = c->reservations || ho.has_rid || ho.has_rt;
    }
    c->types.push_back(std::move(h));
  }
  *out = c;
  return KP_OK;
}
uint64_t kp_catalog_seqnum(const kp_catalog* c) { return c ? c->seqnum : 0; }
uint32_t kp_catalog_size(const kp_catalog* c) { return c ? (uint32_t)c->types.size() : 0; }
namespace {
void DropBasesOf(kp_ctx* ctx, const kp_catalog* c);
}
// A catalogue may be destroyed while plans prepared on it still exist: they (and the ctx's cached bases, which are
// dropped here) see its alive token cleared and return KP_E_INVAL instead of reading it.
void kp_catalog_destroy(kp_catalog* c) {
  if (!c) return;
  std::unique_lock<std::recursive_mutex> lock;
  if (c->ctx) {
    lock = std::unique_lock<std::recursive_mutex>(c->ctx->mu);
    DropBasesOf(c->ctx, c);
  }
  *c->alive = false;
  if (lock.owns_lock()) lock.unlock();  // (the delete may drop the context's last reference)
  delete c;
}

// UnavailableOfferings.MarkUnavailable + SeqNum bump (R:pkg/cache/unavailableofferings.go:66-92) on the uploaded
// offerings; the next prepare (or kp_filter_refresh) rebuilds Available exactly as createOfferings does
// (R:offering.go:115-147). Validated in full before anything changes.
int32_t kp_catalog_update_offerings(kp_catalog* c, const kp_offering_update* ups, uint32_t n, uint64_t seqnum) {
  if (!c || (!ups && n)) return fail(KP_E_INVAL, "null argument");
  // serialized with every prepare / refresh / run of the catalogue's context (they read c->types)
  std::unique_lock<std::recursive_mutex> lock;
  if (c->ctx) lock = std::unique_lock<std::recursive_mutex>(c->ctx->mu);
  auto match = [](const HostOffering& o, const kp_offering_update& u) {
    if (o.ct != (u.capacity_type ? u.capacity_type : "")) return false;
    if (u.reservation_id && !(o.has_rid && o.rid == u.reservation_id)) return false;
    return u.zone ? (o.has_zone && o.zone == u.zone) : !o.has_zone;
  };
  for (uint32_t i = 0; i < n; i++) {
    if (ups[i].type >= c->types.size())
      return fail(KP_E_INVAL, "update %u: type %u of %zu", i, ups[i].type, c->types.size());
    bool any = false;
    for (auto& o : c->types[ups[i].type].offs) {
      if (!match(o, ups[i])) continue;
      any = true;
      // a reserved offering is Available only with capacity left (R:offering.go:178 ReservationCapacity != 0 &&
      // zone in itZones): an update giving capacity 0 with available set names a state upstream cannot reach
      if ((o.has_rid || o.ct == "reserved") && ups[i].reservation_capacity == 0 && ups[i].available)
        return fail(KP_E_INVAL, "update %u: reserved offering of type %u available with reservation capacity 0", i,
                    ups[i].type);
    }
    if (!any) return fail(KP_E_INVAL, "update %u names no offering of type %u", i, ups[i].type);
  }
  for (uint32_t i = 0; i < n; i++)
    for (auto& o : c->types[ups[i].type].offs)
      if (match(o, ups[i])) {
        o.available = ups[i].available != 0;
        if (!std::isnan(ups[i].price)) o.price = ups[i].price;
        if (ups[i].reservation_capacity >= 0) o.rcap = ups[i].reservation_capacity;
      }
  c->seqnum = seqnum;
  return KP_OK;
}

namespace {
int64_t EniLimitedPods(const kp_ec2_info* info, int reserved) {  // ENILimitedPods (R:types.go:461-475)
  int64_t usable = std::max<int64_t>((int64_t)info->max_enis - reserved, 0);
  return usable == 0 ? 0 : usable * ((int64_t)info->ipv4_per_eni - 1) + 2;
}
void SetRes(kp_resource_list* l, int r, int64_t v) {
  l->milli[r] = v;
  l->present |= 1u << r;
}
struct FamilyFlags;
int64_t PodsOf(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc);
int64_t MemoryBytes(const kp_options* opts, const kp_ec2_info* info) {  // memory() (R:types.go:337-347)
  int64_t mib = info->memory_mib;
  if (info->arch && strcmp(info->arch, "arm64") == 0) mib -= 64;  // Graviton CMA
  const int64_t ovMiB = (int64_t)std::ceil((double)(mib * 1048576ll) * opts->vm_memory_overhead_percent / 1024 / 1024);
  return (mib - ovMiB) * 1048576ll;
}
// An AMI family's FeatureFlags and its default ephemeral volume (no blockDeviceMappings on the nodeclass):
// DefaultFamily (AL2023, AL2, Custom) R:amifamily/resolver.go:110-117; Bottlerocket :126-132 (/dev/xvdb, DefaultEBS);
// Windows windows.go:101-108 (/dev/sda1, 50Gi); the others DefaultEBS 20Gi (resolver.go:39-43).
struct FamilyFlags {
  bool eni_memory, pods_per_core, eviction_soft, eni_density, windows;
  int64_t storage_bytes;
};
// ephemeralStorage (R:pkg/providers/instancetype/types.go:349-385), in bytes: instanceStorePolicy RAID0 -> the
// instance store's total size ("%dG"); else the first root-volume BDM with a volumeSize; else for Custom the last
// BDM's volumeSize or DefaultEBS (20Gi), for the other families the first BDM on the family's ephemeral device
// (R:amifamily al2023.go:106-108, al2.go:114-116, bottlerocket.go:110-112, windows.go:97-99) with a volumeSize;
// else the family's default BDM on that device (Bottlerocket :95-108 and the DefaultEBS families 20Gi, Windows
// :88-95 50Gi, Custom none: DefaultEBS).
int64_t EphemeralBytes(const kp_ec2_info* info, const kp_nodeclass* nc) {
  const int64_t kDefaultEBS = 20ll << 30;
  const int f = nc ? nc->ami_family : KP_AMI_AL2023;
  const bool windows = f == KP_AMI_WINDOWS2019 || f == KP_AMI_WINDOWS2022;
  if (nc && nc->instance_store_policy == KP_INSTANCE_STORE_RAID0) {
    const int64_t gb = info->instance_storage_gb > 0 ? info->instance_storage_gb : info->local_nvme_gb;
    if (gb > 0) return gb * 1000000000ll;
  }
  if (nc && nc->n_block_device_mappings && nc->block_device_mappings) {
    const kp_block_device_mapping* b = nc->block_device_mappings;
    const uint32_t n = nc->n_block_device_mappings;
    for (uint32_t i = 0; i < n; i++)
      if (b[i].root_volume) {  // lo.Find: the first root volume only
        if (b[i].volume_size >= 0) return b[i].volume_size;
        break;
      }
    if (f == KP_AMI_CUSTOM) return b[n - 1].volume_size >= 0 ? b[n - 1].volume_size : kDefaultEBS;
    const char* dev = f == KP_AMI_BOTTLEROCKET ? "/dev/xvdb" : windows ? "/dev/sda1" : "/dev/xvda";
    for (uint32_t i = 0; i < n; i++)
      if (b[i].device_name && strcmp(b[i].device_name, dev) == 0) {
        if (b[i].volume_size >= 0) return b[i].volume_size;
        break;
      }
  }
  return windows ? 50ll << 30 : kDefaultEBS;
}

FamilyFlags Family(const kp_nodeclass* nc) {
  const int f = nc ? nc->ami_family : KP_AMI_AL2023;
  if (f == KP_AMI_BOTTLEROCKET) return {false, false, false, true, false, 20ll << 30};
  if (f == KP_AMI_WINDOWS2019 || f == KP_AMI_WINDOWS2022) return {false, true, true, false, true, 50ll << 30};
  return {true, true, true, true, false, 20ll << 30};
}

// pods() (R:types.go:553-569): maxPods, else ENI-limited when the family supports it, else 110; then podsPerCore
int64_t PodsOf(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc) {
  const FamilyFlags fam = Family(nc);
  int64_t pods = (nc && nc->max_pods >= 0) ? nc->max_pods : fam.eni_density ? EniLimitedPods(info, opts->reserved_enis) : 110;
  if (nc && nc->pods_per_core > 0 && fam.pods_per_core) pods = std::min<int64_t>((int64_t)nc->pods_per_core * info->vcpu, pods);
  return pods;
}

// computeEvictionSignal (R:types.go:571-598) in milli-units: a percentage p of the capacity (100% disables the
// threshold) as ceil(capacity / 100 * p) whole units, else the quantity itself.
int64_t EvictionSignalMilli(int64_t capacity_units, const kp_eviction_value& v) {
  if (!v.is_percent) return v.milli;
  const double p = v.percent == 100.0 ? 0.0 : v.percent;
  return (int64_t)std::ceil((double)capacity_units / 100 * p) * 1000;
}
}  // namespace

int32_t kp_instance_type_overhead(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc,
                                  kp_resource_list* kube, kp_resource_list* sys, kp_resource_list* ev) {
  if (!opts || !info || !kube || !sys || !ev) return fail(KP_E_INVAL, "null argument");
  const kp_kubelet* kl = nc ? nc->kubelet : nullptr;
  memset(kube, 0, sizeof *kube);
  memset(sys, 0, sizeof *sys);
  memset(ev, 0, sizeof *ev);
  const FamilyFlags fam = Family(nc);
  const int64_t kStorageBytes = EphemeralBytes(info, nc);
  // kubeReservedResources: UsesENILimitedMemoryOverhead -> memory from ENILimitedPods(info, 0), else from pods(); the
  // CPU ranges accumulate with a truncation per range; then the user's keys replace the computed ones (lo.Assign)
  SetRes(kube, KP_RES_MEMORY, (11 * (fam.eni_memory ? EniLimitedPods(info, 0) : PodsOf(opts, info, nc)) + 255) * 1048576ll * 1000ll);
  SetRes(kube, KP_RES_EPHEMERAL_STORAGE, (1ll << 30) * 1000);
  const struct {
    int64_t s, e;
    double p;
  } rg[4] = {{0, 1000, 0.06}, {1000, 2000, 0.01}, {2000, 4000, 0.005}, {4000, 1ll << 31, 0.0025}};
  const int64_t cpuM = (int64_t)info->vcpu * 1000;
  int64_t cpuOverhead = 0;
  for (auto& x : rg)
    if (cpuM >= x.s) cpuOverhead += (int64_t)((double)(cpuM < x.e ? cpuM - x.s : x.e - x.s) * x.p);
  SetRes(kube, KP_RES_CPU, cpuOverhead);
  if (kl)
    for (int r = 0; r < KP_NUM_RESOURCES; r++)
      if (kl->kube_reserved.present & (1u << r)) SetRes(kube, r, kl->kube_reserved.milli[r]);
  // systemReservedResources: exactly the user's map
  if (kl)
    for (int r = 0; r < KP_NUM_RESOURCES; r++)
      if (kl->system_reserved.present & (1u << r)) SetRes(sys, r, kl->system_reserved.milli[r]);
  // evictionThreshold: defaults, then MaxResources over the signal maps (hard, then soft), assigned over them
  SetRes(ev, KP_RES_MEMORY, 100ll * 1048576ll * 1000ll);
  SetRes(ev, KP_RES_EPHEMERAL_STORAGE, (int64_t)std::ceil((double)kStorageBytes / 100 * 10) * 1000);
  if (kl) {
    const int64_t memBytes = MemoryBytes(opts, info);
    kp_resource_list ov{};
    auto fold = [&](const kp_eviction_value& mem, const kp_eviction_value& fs) {
      if (mem.set) {
        const int64_t v = EvictionSignalMilli(memBytes, mem);
        if (!(ov.present & (1u << KP_RES_MEMORY)) || v > ov.milli[KP_RES_MEMORY]) SetRes(&ov, KP_RES_MEMORY, v);
      }
      if (fs.set) {
        const int64_t v = EvictionSignalMilli(kStorageBytes, fs);
        if (!(ov.present & (1u << KP_RES_EPHEMERAL_STORAGE)) || v > ov.milli[KP_RES_EPHEMERAL_STORAGE])
          SetRes(&ov, KP_RES_EPHEMERAL_STORAGE, v);
      }
    };
    if (kl->has_eviction_hard) fold(kl->hard_memory_available, kl->hard_nodefs_available);
    if (kl->has_eviction_soft && fam.eviction_soft) fold(kl->soft_memory_available, kl->soft_nodefs_available);
    for (int r = 0; r < KP_NUM_RESOURCES; r++)
      if (ov.present & (1u << r)) SetRes(ev, r, ov.milli[r]);
  }
  return KP_OK;
}

// instancetype.NewInstanceType capacity + Overhead.Total() for the nodeclass's AMI family (R:types.go:123-155, 313-598).
int32_t kp_instance_type_resolve(const kp_options* opts, const kp_ec2_info* info, const kp_nodeclass* nc,
                                 kp_resource_list* capacity, kp_resource_list* overhead) {
  if (!opts || !info || !capacity || !overhead) return fail(KP_E_INVAL, "null argument");
  memset(capacity, 0, sizeof *capacity);
  memset(overhead, 0, sizeof *overhead);
  SetRes(capacity, KP_RES_CPU, (int64_t)info->vcpu * 1000);
  SetRes(capacity, KP_RES_MEMORY, MemoryBytes(opts, info) * 1000);
  const FamilyFlags fam = Family(nc);
  SetRes(capacity, KP_RES_EPHEMERAL_STORAGE, EphemeralBytes(info, nc) * 1000);
  SetRes(capacity, KP_RES_PODS, PodsOf(opts, info, nc) * 1000);
  SetRes(capacity, KP_RES_POD_ENI, (info->in_limits_table && info->trunking) ? (int64_t)info->branch_enis * 1000 : 0);
  const string gm = info->gpu_manufacturer ? info->gpu_manufacturer : "";
  SetRes(capacity, KP_RES_NVIDIA_GPU, gm == "nvidia" ? info->gpu_count * 1000ll : 0);
  SetRes(capacity, KP_RES_AMD_GPU, gm == "amd" ? info->gpu_count * 1000ll : 0);
  SetRes(capacity, KP_RES_NEURON, (int64_t)info->neuron_devices * 1000);
  SetRes(capacity, KP_RES_NEURONCORE, (int64_t)info->neuron_devices * info->neuron_cores_per_device * 1000);
  SetRes(capacity, KP_RES_GAUDI, gm == "habana" ? info->gpu_count * 1000ll : 0);
  SetRes(capacity, KP_RES_EFA, (int64_t)info->efa * 1000);
  // Windows: the os requirement is windows only for amd64 types (getOS), which then get PrivateIPv4Address
  if (fam.windows && info->arch && strcmp(info->arch, "amd64") == 0)
    SetRes(capacity, KP_RES_PRIVATE_IPV4, info->in_limits_table ? ((int64_t)info->ipv4_per_eni - 1) * 1000 : 0);
  kp_resource_list parts[3];
  int32_t rc = kp_instance_type_overhead(opts, info, nc, &parts[0], &parts[1], &parts[2]);
  if (rc != KP_OK) return rc;
  for (auto& l : parts)  // InstanceTypeOverhead.Total(): resources.Merge of the three lists
    for (int r = 0; r < KP_NUM_RESOURCES; r++)
      if (l.present & (1u << r)) SetRes(overhead, r, overhead->milli[r] + l.milli[r]);
  return KP_OK;
}

}  // extern "C"

// ==================================================================================================
// Solve
// ==================================================================================================
namespace {

struct TaintT {
  string key, value;
  int effect;
  bool operator<(const TaintT& o) const { return std::tie(key, value, effect) < std::tie(o.key, o.value, o.effect); }
};

// The part of a Solve's compiled form that depends only on the catalogues (identity + seqnum) and the NodePools:
// the string dictionary, every catalogue SoA, the offering classes and the NodeClaimTemplates (upstream
// NewScheduler's per-template pre-filter). It is built on a cache miss and kept resident (host + device) in the
// kp_ctx across Solves, keyed by that fingerprint (R:pkg/providers/instancetype/instancetype.go:225-237 cacheKey:
// the reference likewise rebuilds its InstanceType list only when a seqnum changes). A Solve whose pods or nodes
// name a label key or value the dictionary lacks triggers a rebuild that adds them (the dictionary only grows).
// Device offsets of one catalogue's arrays inside an upload blob.
struct CatOffsets {
  size_t TM, DNE, NOKEY, alloc, cap, nonneg, fit_vals, fit_n, fit_mask, cls, offer, price, price_cm, price_sub, rank, code, multi, custom;
};

struct SolveBase {
  Dict d;
  int TW = 1, C = 0;
  vector<HostCat> cats;
  vector<OfferClass> classes;
  // templates (weight desc, name asc; pools whose requirements filter out every type are skipped)
  vector<int> tmpl_nodepool;          // index into kp_solve_in.nodepools
  vector<KReqs> tmpl_reqs;
  vector<int32_t> tmpl_taintset, tmpl_catalog;
  vector<uint64_t> tmpl_X;
  vector<int64_t> tmpl_daemon;
  vector<vector<TaintT>> tsets;       // the NodePools' taint sets in id order
  vector<int> np_taintset;            // per input NodePool
  // the NodePools as the templates need them (input order; np_order = weight desc, name asc), so that an ICE update
  // can rebuild the templates' options without the caller's kp_solve_in
  vector<KReqs> np_q;
  vector<int32_t> np_catalog;
  vector<int> np_order;
  vector<int64_t> np_daemon;          // [n_nodepools][NRES]
  vector<const kp_catalog*> catalogs; // the catalogues compiled in (caller-owned; see alive)
  vector<std::shared_ptr<bool>> alive; // their kp_catalog::alive tokens: a destroyed one makes the base unusable
  vector<uint64_t> seqnums;           // their seqnums the offering arrays reflect
  string ident;                       // cache fingerprint without the seqnums
  string key;                         // cache fingerprint: ident + seqnums
  uint64_t version = 0;               // bumped by every in-place offering refresh (RefreshOfferings)
  // device copy (Solve plans): dict, parsed integers, catalogue SoA + descriptors, templates
  DevBuf dev;
  bool on_device = false;
  size_t o_dict = 0, o_vint = 0, o_cats = 0, o_treqs = 0, o_tts = 0, o_tcat = 0, o_tX = 0, o_tdm = 0;
  vector<CatOffsets> coffs;
  double build_ms = 0;
  // capacity reservations (NewReservationManager): the reserved offering classes (one per reservation id) and the
  // least ReservationCapacity the NodePools' catalogues report for each
  uint64_t res_cls = 0;
  vector<int32_t> res_cap0;
};

// NewReservationManager's starting capacities (UP reservationmanager.go: the least ReservationCapacity any NodePool's
// instance types report for an id). Requires one class per reservation id (a reservation is one type in one zone).
int32_t ReservationTables(SolveBase& b) {
  b.res_cls = 0;
  b.res_cap0.assign(KP_MAX_CLASSES, 0);
  const int ct = b.d.key(kCapType), res = ct >= 0 ? b.d.bit(ct, "reserved") : -1;
  if (res < 0) return KP_OK;
  map<int, int> rid_class;
  for (int c = 0; c < b.C; c++) {
    if (b.classes[c].ct_bit != res) continue;
    if (b.classes[c].rid_bit < 0) return fail(KP_E_UNSUPPORTED, "reserved offering class without a reservation id");
    if (!rid_class.emplace(b.classes[c].rid_bit, c).second)
      return fail(KP_E_UNSUPPORTED, "one capacity reservation in two offering classes");
    b.res_cls |= 1ull << c;
    b.res_cap0[c] = INT32_MAX;
  }
  if (!b.res_cls) return KP_OK;
  map<ClassKey, int> classes;
  for (int c = 0; c < b.C; c++) classes[KeyOfClass(b.classes[c])] = c;
  for (int np = 0; np < (int)b.np_catalog.size(); np++)
    for (auto& t : b.catalogs[b.np_catalog[np]]->types)
      for (auto& o : t.offs) {
        const int c = classes.at(ClassOf(b.d, o));
        if ((b.res_cls >> c) & 1) b.res_cap0[c] = std::min(b.res_cap0[c], std::max(o.rcap, 0));
      }
  for (int c = 0; c < b.C; c++)
    if (b.res_cap0[c] == INT32_MAX) b.res_cap0[c] = 0;  // only in catalogues no NodePool uses
  return KP_OK;
}

struct Compiled {
  kp_overrides ov{};  // the context's overrides at compile time (CompileSolve with a ctx)
  std::shared_ptr<SolveBase> B = std::make_shared<SolveBase>();
  bool base_hit = false;              // the base came from the ctx cache
  bool base_refreshed = false;        // ... after an in-place offering refresh (a new catalogue seqnum)
  vector<uint32_t> tmpl_limit_present;
  vector<int64_t> tmpl_remaining;
  // shapes
  vector<int32_t> shape_level_base, shape_nlevels;
  int32_t cont_hint = 0;  // most queue neighbours share their shape: the fast lane with its continuation round
  vector<KReqs> shape_reqs;
  vector<uint64_t> shape_negop, shape_tolerates;  // per shape-level (tolerations change at the PreferNoSchedule level)
  vector<char> sl_pns;                             // per shape-level: toleratePreferNoScheduleTaints' level
  vector<int64_t> shape_requests;
  vector<uint64_t> pvp;
  vector<int32_t> pvp_base, pvp_slot, pvp_n;  // pvp_n: rows of catalogue 0 per shape-level
  // existing (sorted)
  vector<int> ex_input;
  vector<KReqs> ex_reqs;
  vector<int32_t> ex_taintset;
  vector<int64_t> ex_available, ex_requests;
  // host ports (HostPortUsage): conflict / add masks per shape over the batch's port bits, used bits per node
  vector<uint64_t> shape_hp_conf, shape_hp_add, ex_hp;
  bool hp_any = false;
  // pods
  vector<int32_t> pod_shape, queue;
  // topology spread (TopologyTypeSpread groups; see SolveArgs)
  int G = 0, GH = 0, TK = 0;
  vector<int32_t> tg_key, tg_row, tg_maxskew, tg_mindom, tg_aff, tg_term_base, tg_nterm;
  vector<uint64_t> tg_filt_tol, tg_reg, tg_terms_negop;
  vector<KReqs> tg_terms;
  vector<int32_t> tg_cnt;    // [G][64]
  vector<int32_t> tg_live;   // [G] 1: the group exists (NewTopology, or a Topology.Update made it); Record skips others
  vector<uint8_t> hcnt0;     // [GH][E]
  vector<int32_t> shape_rec_base, shape_rec_n, rec_list;
  vector<int32_t> sl_own_base, sl_own_n, own_group, own_self;
  vector<int32_t> sl_fast_topo;  // [SL] 1: the fast lane may place the level's pods (append path; see CompileTopology)
  vector<int32_t> rec_aux;       // per rec_list entry: the group's hostname row, else -1 - its key's slot
  vector<int32_t> own_rec;  // [O][8] static part of an owned group: group, self, key, maxSkew, minDomains, row, key slot, 0
  vector<uint64_t> own_pd, sl_topo_keys;
  vector<int32_t> tkey_slot;  // [64]
  vector<int32_t> tk_keys;    // [TK]
  vector<uint8_t> ex_tcode;   // [TK][E]
  // What each existing node (input index) contributes to the topology state, recorded by CompileTopology when
  // track_nodes is set: the batched general-path simulations (GeneralBatch) remove a subset's nodes from it.
  bool track_nodes = false;
  vector<vector<int32_t>> node_cnt;  // [n_existing] tg_cnt entries (g * 64 + ordinal), one per bound pod counted
  vector<vector<int32_t>> node_reg;  // [n_existing] (g * 64 + ordinal): a domain the node registers in dictionary-key group g
  vector<vector<int32_t>> node_hrec; // [n_existing] hostname-row groups a bound pod on the node was recorded into
  vector<vector<int32_t>> node_inv;  // [n_existing] inverse anti-affinity groups a bound pod on the node owns
  vector<uint64_t> tg_reg_static;    // [G] domains registered without any existing node (NodePool / type offerings)
  vector<int32_t> tg_hrec_total, tg_inv_total;  // [G]
  vector<vector<int32_t>> shape_l0;  // [S] the spread groups each shape makes at level 0 (NewTopology, if it has pods)
  vector<char> tg_spread;            // [G] 1: a topology-spread group
  vector<vector<int32_t>> tg_unreg;  // [G] hostname spread groups: positions (sorted order) unregistered (255) when the
                                     // group is created not live
};

// Requirements.Compatible(A, B, allowUndefinedWellKnown) on the host encoding.
bool HostCompatible(const Dict& d, const KReqs& A, const KReqs& B, bool allow) {
  const uint64_t negB = NegOp(d, B), negA = NegOp(d, A);
  uint64_t undef = B.present & ~A.present & ~negB;
  if (allow) undef &= ~d.dd.wellknown;
  if (undef) return false;
  KReqs m = A;
  HostAdd(d, m, B);
  const uint64_t shared = A.present & B.present;
  for (int k = 0; k < d.dd.K; k++) {
    if (!((shared >> k) & 1)) continue;
    const bool empty = !((m.compl_ >> k) & 1) && !KeyNonEmptyVals(d, m, k);  // Len() == 0
    if (empty && !(((negA & negB) >> k) & 1)) return false;
  }
  return true;
}

// Semantic canonical form of a requirement set (identity of a topology node filter).
string KCanon(const Dict& d, const KReqs& q) {
  string o;
  for (int k = 0; k < d.dd.K; k++) {
    if (!((q.present >> k) & 1)) continue;
    const bool bnd = k < KP_MAX_BOUND_KEYS;
    o += std::to_string(k) + ((q.compl_ >> k) & 1 ? "!" : "=");
    for (int i = 0; i < nwords(d, k); i++) o += std::to_string(q.vals[kw(d, k, i)]) + ",";
    if (bnd && ((q.hgt >> k) & 1)) o += ">" + std::to_string(q.gt[k]);
    if (bnd && ((q.hlt >> k) & 1)) o += "<" + std::to_string(q.lt[k]);
    if (bnd && ((q.hmin >> k) & 1)) o += "#" + std::to_string(q.minv[k]);
    o += ";";
  }
  return o;
}

// metav1.LabelSelector.Matches (nil selects nothing)
bool SelectorMatches(const kp_label_selector& sel, const std::map<string, string>& labels) {
  if (sel.is_nil) return false;
  for (uint32_t i = 0; i < sel.n_match_labels; i++) {
    auto it = labels.find(sel.match_labels[i].key ? sel.match_labels[i].key : "");
    if (it == labels.end() || it->second != (sel.match_labels[i].value ? sel.match_labels[i].value : "")) return false;
  }
  for (uint32_t i = 0; i < sel.n_match_expressions; i++) {
    const kp_selector_requirement& r = sel.match_expressions[i];
    auto it = labels.find(r.key ? r.key : "");
    const bool has = it != labels.end();
    bool in = false;
    for (uint32_t j = 0; has && j < r.n_values && !in; j++) in = it->second == (r.values[j] ? r.values[j] : "");
    switch (r.op) {
      case KP_SEL_IN:
        if (!in) return false;
        break;
      case KP_SEL_NOT_IN:
        if (in) return false;
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
string SelectorCanon(const kp_label_selector& sel) {
  if (sel.is_nil) return "nil";
  vector<string> parts;
  for (uint32_t i = 0; i < sel.n_match_labels; i++)
    parts.push_back(string(sel.match_labels[i].key) + "/0," + (sel.match_labels[i].value ? sel.match_labels[i].value : ""));
  for (uint32_t i = 0; i < sel.n_match_expressions; i++) {
    const kp_selector_requirement& r = sel.match_expressions[i];
    std::set<string> vs;
    for (uint32_t j = 0; j < r.n_values; j++) vs.insert(r.values[j] ? r.values[j] : "");
    string x = string(r.key) + "/" + std::to_string(r.op);
    for (auto& v : vs) x += "," + v;
    parts.push_back(x);
  }
  std::sort(parts.begin(), parts.end());
  string o;
  for (auto& x : parts) o += x + ";";
  return o;
}
std::map<string, string> LabelMap(const kp_label* l, uint32_t n) {
  std::map<string, string> m;
  for (uint32_t i = 0; i < n; i++) m[l[i].key ? l[i].key : ""] = l[i].value ? l[i].value : "";
  return m;
}

// Topology spread groups (upstream NewTopology / TopologyGroup / countDomains / buildDomainGroups), in the
// device encoding: one group per distinct (key, maxSkew, namespace, selector, node filter, policies) in order
// of first appearance over the pods; dictionary-key groups keep a count per value ordinal + a registered-
// domain mask, hostname groups a saturating u8 count per node (existing positions, then NodeClaims).
// A pod's podAntiAffinity terms in one list: required terms, then preferred ones (spec order).
// A pod's inter-pod terms in one list: required anti-affinity, preferred anti-affinity, required affinity, preferred
// affinity (spec order within each). *aff: the term is a podAffinity term.
uint32_t PodTermCount(const kp_pod_shape& sh) {
  return sh.n_required_anti_affinity + sh.n_preferred_anti_affinity + sh.n_required_affinity + sh.n_preferred_affinity;
}
const kp_pod_affinity_term* PodTermAt(const kp_pod_shape& sh, int a, bool* aff = nullptr) {
  const uint32_t n[4] = {sh.n_required_anti_affinity, sh.n_preferred_anti_affinity, sh.n_required_affinity,
                         sh.n_preferred_affinity};
  const kp_pod_affinity_term* p[4] = {sh.required_anti_affinity, sh.preferred_anti_affinity, sh.required_affinity,
                                      sh.preferred_affinity};
  for (int i = 0; i < 4; i++) {
    if (a < (int)n[i]) {
      if (aff) *aff = i >= 2;
      return &p[i][a];
    }
    a -= (int)n[i];
  }
  return nullptr;
}
int32_t CheckAntiTerm(const kp_pod_affinity_term& t, const char* who, uint32_t i) {
  if (!t.topology_key || !t.topology_key[0]) return fail(KP_E_INVAL, "%s %u: pod (anti-)affinity without topologyKey", who, i);
  return KP_OK;
}

// HostPortUsage.Conflicts as bit masks. Bits: U(g) per (protocol, port) group g some unspecified-IP entry names,
// S(g, ip) per specific entry. An entry (g, unspecified) conflicts with every used bit of g and adds U(g); an
// entry (g, ip) conflicts with U(g) and S(g, ip) and adds S(g, ip) — HostPort.Matches (same protocol and port, and
// an unspecified IP on either side or equal IPs). A node's used bits only grow, so a conflict is permanent.
int32_t EncodeHostPorts(const vector<vector<HostPortKey>>& shapes, const vector<vector<HostPortKey>>& nodes,
                        Compiled& cp) {
  std::map<std::pair<int, int>, int> ubit;                               // group -> U bit
  std::map<std::pair<std::pair<int, int>, std::array<uint8_t, 16>>, int> sbit;  // (group, ip) -> S bit
  std::map<std::pair<int, int>, uint64_t> gmask;                         // every bit of a group
  int nb = 0;
  auto visit = [&](const vector<HostPortKey>& v) {
    for (auto& k : v) {
      const auto g = std::make_pair(k.proto, k.port);
      if (k.unspec) {
        if (!ubit.count(g)) ubit[g] = nb++;
      } else if (!sbit.count({g, k.ip})) {
        sbit[{g, k.ip}] = nb++;
      }
    }
  };
  for (auto& v : shapes) visit(v);
  for (auto& v : nodes) visit(v);
  if (nb > 64) return fail(KP_E_UNSUPPORTED, "%d distinct host port entries (max 64)", nb);
  for (auto& kv : ubit) gmask[kv.first] |= 1ull << kv.second;
  for (auto& kv : sbit) gmask[kv.first.first] |= 1ull << kv.second;
  auto masks = [&](const vector<HostPortKey>& v, uint64_t* conf, uint64_t* add) {
    *conf = *add = 0;
    for (auto& k : v) {
      const auto g = std::make_pair(k.proto, k.port);
      auto u = ubit.find(g);
      const uint64_t ub = u == ubit.end() ? 0 : 1ull << u->second;
      if (k.unspec) {
        *conf |= gmask[g];
        *add |= ub;
      } else {
        const uint64_t sb = 1ull << sbit[{g, k.ip}];
        *conf |= ub | sb;
        *add |= sb;
      }
    }
  };
  cp.shape_hp_conf.assign(shapes.size(), 0);
  cp.shape_hp_add.assign(shapes.size(), 0);
  for (size_t i = 0; i < shapes.size(); i++) masks(shapes[i], &cp.shape_hp_conf[i], &cp.shape_hp_add[i]);
  cp.ex_hp.assign(nodes.size(), 0);
  for (size_t i = 0; i < nodes.size(); i++) {
    uint64_t c;
    masks(nodes[i], &c, &cp.ex_hp[i]);
  }
  cp.hp_any = nb > 0;
  return KP_OK;
}

// the toleration Preferences.toleratePreferNoScheduleTaints appends, and whether the pod already carries it
// (corev1 Toleration.MatchToleration: equal key, operator, value and effect)
const kp_toleration kPnsToleration = {"", "", KP_TOL_EXISTS, KP_EFFECT_PREFER_NO_SCHEDULE};
bool HasPnsToleration(const kp_pod_shape& sh) {
  for (uint32_t j = 0; j < sh.n_tolerations; j++) {
    const kp_toleration& t = sh.tolerations[j];
    if ((!t.key || !t.key[0]) && (!t.value || !t.value[0]) && t.op == KP_TOL_EXISTS &&
        t.effect == KP_EFFECT_PREFER_NO_SCHEDULE)
      return true;
  }
  return false;
}

// kp_overrides.host_timing: host compile phases on stderr (diagnostics only)
struct PhaseTimer {
  bool on = g_host_timing.load(std::memory_order_relaxed);
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[kp compile] %-22s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

int32_t CompileTopology(const kp_solve_in* in, Compiled& cp, const vector<vector<RawReqs>>& strict_levels,
                        const vector<vector<vector<int>>>& spread_levels, const vector<int>& np_taintset,
                        const vector<vector<vector<RawReqs>>>& filter_levels) {
  const Dict& d = cp.B->d;
  const int E = (int)cp.ex_input.size();
  cp.tkey_slot.assign(KP_MAX_KEYS, -1);
  cp.shape_rec_base.assign(in->n_shapes, 0);
  cp.shape_rec_n.assign(in->n_shapes, 0);
  const size_t SL = cp.shape_reqs.size();
  cp.sl_own_base.assign(SL, 0);
  cp.sl_own_n.assign(SL, 0);
  cp.sl_topo_keys.assign(SL, 0);
  cp.sl_fast_topo.assign(SL, 1);
  bool any = false;
  for (uint32_t s = 0; s < in->n_shapes; s++)
    any |= in->shapes[s].n_topology_spread + PodTermCount(in->shapes[s]) > 0;
  for (uint32_t b = 0; b < in->n_bound_pods; b++) {
    for (uint32_t j = 0; j < in->bound_pods[b].n_anti_affinity; j++) {
      const int32_t rc = CheckAntiTerm(in->bound_pods[b].anti_affinity[j], "bound pod", b);
      if (rc) return rc;
    }
    any |= in->bound_pods[b].n_anti_affinity > 0;
  }
  if (!any) return KP_OK;
  PhaseTimer pt;
  if (cp.track_nodes) {
    cp.node_cnt.assign(in->n_existing, {});
    cp.node_reg.assign(in->n_existing, {});
    cp.node_hrec.assign(in->n_existing, {});
    cp.node_inv.assign(in->n_existing, {});
    cp.shape_l0.assign(in->n_shapes, {});
  }
  vector<int> ex_pos(in->n_existing);
  for (int e = 0; e < E; e++) ex_pos[cp.ex_input[e]] = e;
  vector<KReqs> node_reqs(in->n_existing);
  for (uint32_t i = 0; i < in->n_existing; i++) node_reqs[i] = cp.ex_reqs[ex_pos[i]];
  // the existing nodes' value of one label key (LabelMap's: the last entry wins; nullptr: no such label), computed
  // once per key that some group reads (a few keys against thousands of nodes)
  std::unordered_map<string, vector<const char*>> node_kv;
  auto node_vals = [&](const string& key) -> const vector<const char*>& {
    auto it = node_kv.find(key);
    if (it != node_kv.end()) return it->second;
    vector<const char*> v(in->n_existing, nullptr);
    for (uint32_t i = 0; i < in->n_existing; i++) {
      const kp_existing_node& e = in->existing[i];
      for (uint32_t j = 0; j < e.n_labels; j++)
        if (key == (e.labels[j].key ? e.labels[j].key : "")) v[i] = e.labels[j].value ? e.labels[j].value : "";
    }
    return node_kv.emplace(key, std::move(v)).first->second;
  };
  // ... and its value ordinal for a dictionary key k (-1: no such label)
  std::unordered_map<int, vector<int>> node_ko;
  auto node_ords = [&](int k) -> const vector<int>& {
    auto it = node_ko.find(k);
    if (it != node_ko.end()) return it->second;
    const vector<const char*>& v = node_vals(d.keys[k]);
    vector<int> o(in->n_existing, -1);
    for (uint32_t i = 0; i < in->n_existing; i++)
      if (v[i]) o[i] = d.bit(k, v[i]) - k * 64;
    return node_ko.emplace(k, std::move(o)).first->second;
  };
  // buildDomainGroups for one key: value ordinal -> taint sets of the NodePools offering it
  std::map<int, vector<uint64_t>> domain_tsets;  // key -> [64] taint-set masks
  auto domains_of = [&](int k) -> const vector<uint64_t>& {
    auto it = domain_tsets.find(k);
    if (it != domain_tsets.end()) return it->second;
    vector<uint64_t> m(64, 0);
    auto insert = [&](const KReqs& r, int ts) {
      if (!((r.present >> k) & 1) || ((r.compl_ >> k) & 1)) return;  // Operator() == In
      uint64_t v = r.vals[k];
      while (v) {
        const int b = __builtin_ctzll(v);
        v &= v - 1;
        m[b] |= 1ull << ts;
      }
    };
    for (uint32_t i = 0; i < in->n_nodepools; i++) {
      const kp_nodepool& np = in->nodepools[i];
      const HostCat& hc = cp.B->cats[np.catalog];
      if (hc.T == 0) continue;
      RawReqs base_raw = ParseReqs(np.requirements);
      RawReqs l = LabelReqs(np.labels, np.n_labels, false);
      base_raw.insert(base_raw.end(), l.begin(), l.end());
      const KReqs base = Compile(d, base_raw);
      for (int t = 0; t < hc.T; t++) {
        KReqs r = base;
        HostAdd(d, r, hc.treqs[t]);
        insert(r, np_taintset[i]);
      }
      insert(base, np_taintset[i]);
    }
    return domain_tsets[k] = m;
  };
  // bound pods grouped by (namespace, labels): deployments repeat one label set over many pods
  struct BoundSet {
    string ns;
    std::map<string, string> labels;
    vector<uint32_t> nodes;  // input indices, one entry per bound pod
  };
  vector<BoundSet> bsets;
  // the sets indexed by (namespace, label) and by namespace: a matchLabels selector only tests the sets carrying its
  // first label (index lists are in set order, so a group visits its sets in the order a full scan would)
  std::unordered_map<string, vector<int>> bs_by_label, bs_by_ns;
  {
    std::unordered_map<string, int> idx;  // canonical (namespace, LabelMap) -> set
    vector<std::pair<const char*, const char*>> kv;
    string canon;
    for (uint32_t b = 0; b < in->n_bound_pods; b++) {
      const kp_bound_pod& bp = in->bound_pods[b];
      if (bp.node >= in->n_existing) return fail(KP_E_INVAL, "bound pod %u: node %u", b, bp.node);
      // LabelMap without the map: the entries by key, stable, the last of equal keys kept
      kv.clear();
      for (uint32_t j = 0; j < bp.n_labels; j++)
        kv.push_back({bp.labels[j].key ? bp.labels[j].key : "", bp.labels[j].value ? bp.labels[j].value : ""});
      std::stable_sort(kv.begin(), kv.end(), [](const auto& x, const auto& y) { return strcmp(x.first, y.first) < 0; });
      canon.assign(bp.namespace_ ? bp.namespace_ : "");
      for (size_t j = 0; j < kv.size(); j++) {
        if (j + 1 < kv.size() && strcmp(kv[j].first, kv[j + 1].first) == 0) continue;
        canon += '\x01';
        canon += kv[j].first;
        canon += '\x02';
        canon += kv[j].second;
      }
      auto it = idx.find(canon);
      if (it == idx.end()) {
        const int id = (int)bsets.size();
        it = idx.emplace(canon, id).first;
        const string ns = bp.namespace_ ? bp.namespace_ : "";
        bsets.push_back({ns, LabelMap(bp.labels, bp.n_labels), {}});
        bs_by_ns[ns].push_back(id);
        for (auto& l : bsets.back().labels) bs_by_label[ns + '\x01' + l.first + '\x01' + l.second].push_back(id);
      }
      bsets[it->second].nodes.push_back(bp.node);
    }
  }
  static const vector<int> kNoSets;
  // the bound-pod sets a selector can match in namespace ns (a superset; callers still test SelectorMatches)
  auto sets_for = [&](const kp_label_selector& sel, const string& ns) -> const vector<int>& {
    if (sel.is_nil) return kNoSets;
    if (sel.n_match_labels) {
      auto it = bs_by_label.find(ns + '\x01' + (sel.match_labels[0].key ? sel.match_labels[0].key : "") + '\x01' +
                                 (sel.match_labels[0].value ? sel.match_labels[0].value : ""));
      return it == bs_by_label.end() ? kNoSets : it->second;
    }
    auto it = bs_by_ns.find(ns);
    return it == bs_by_ns.end() ? kNoSets : it->second;
  };
  pt.lap("  topo: labels+bsets");
  std::map<string, int> ids;
  std::map<string, uint64_t> node_domains;
  vector<int> g_shape;  // shape that created the group (its tolerations / filter)
  vector<const kp_topology_spread*> g_spec;
  vector<const kp_label_selector*> g_sel;   // every group: its selector
  vector<std::set<string>> g_nss;           // namespaces it selects in (spread: the owner's)
  vector<char> g_inverse;                   // inverse anti-affinity group (bound pods own it; never recorded)
  // group identity per (shape, spread index)
  vector<vector<int>> sgroup(in->n_shapes);
  vector<char> seen(in->n_shapes, 0);
  // A spread group at relaxation level l of shape s. MakeTopologyNodeFilter: the nodeSelector with each remaining
  // required node-affinity term (ORed); relaxing a term (Preferences.removeRequiredNodeAffinityTerm) changes the
  // filter and so the group identity: Topology.Update then makes a new group, counted from the cluster alone, which
  // exists (is live: records count into it) from that first relaxation on (upstream Topology.Update).
  auto group_of = [&](uint32_t s, int j, int l, bool live) -> int32_t {
    const kp_pod_shape& sh = in->shapes[s];
    const kp_topology_spread& t = sh.topology_spread[j];
    const string key = t.topology_key ? t.topology_key : "";
    const bool aff = t.node_affinity_policy != KP_POLICY_IGNORE, taint = t.node_taints_policy == KP_POLICY_HONOR;
    vector<KReqs> filts;
    for (auto& fr : filter_levels[s][l]) filts.push_back(Compile(d, fr));
    bool nonempty = true;  // an empty term admits every node: the filter is vacuous
    for (auto& f : filts) nonempty = nonempty && f.present != 0;
    string fcanon;
    for (auto& f : filts) fcanon += "[" + KCanon(d, f) + "]";
    string id = key + "|" + std::to_string(t.max_skew) + "|" + (sh.namespace_ ? sh.namespace_ : "") + "|" +
                SelectorCanon(t.selector) + "|" + std::to_string(aff) + std::to_string(taint) + "|" + fcanon;
    const int sl = cp.shape_level_base[s] + l;
    const uint64_t ltol = cp.shape_tolerates[sl];  // the level's tolerations (Relax may have appended one)
    // upstream MakeTopologyNodeFilter keeps the pod's tolerations under every taint policy and TopologyGroup.Hash
    // hashes the whole filter: the tolerations are part of the identity even when the policy ignores them (a pod
    // relaxed to tolerate PreferNoSchedule makes a new group, counted from the cluster alone)
    for (uint32_t i = 0; i < sh.n_tolerations + (cp.sl_pns[sl] ? 1 : 0); i++) {
      const kp_toleration& x = i < sh.n_tolerations ? sh.tolerations[i] : kPnsToleration;
      id += string("(") + (x.key ? x.key : "") + "," + (x.value ? x.value : "") + "," + std::to_string(x.op) + "," +
            std::to_string(x.effect) + ")";
    }
    auto it = ids.find(id);
    if (it != ids.end()) {
      if (live) cp.tg_live[it->second] = 1;
      return it->second;
    }
    const int g = cp.G++;
    ids[id] = g;
    cp.tg_live.push_back(live ? 1 : 0);
    g_shape.push_back((int)s);
    g_spec.push_back(&t);
    g_sel.push_back(&t.selector);
    g_nss.push_back({sh.namespace_ ? sh.namespace_ : ""});
    g_inverse.push_back(0);
    int k = -1, row = -1;
    if (key == kHostname) {
      row = cp.GH++;
    } else {
      k = d.key(key);
      if (k < 0) return fail(KP_E_INVAL, "topology key %s missing from the dictionary", key.c_str()), -1;
      if (d.dd.nval[k] > 64) return fail(KP_E_UNSUPPORTED, "topology key %s has > 64 values", key.c_str()), -1;
      if (cp.tkey_slot[k] < 0) {
        cp.tkey_slot[k] = cp.TK++;
        cp.tk_keys.push_back(k);
      }
    }
    cp.tg_key.push_back(k);
    cp.tg_row.push_back(row);
    cp.tg_maxskew.push_back(t.max_skew);
    cp.tg_mindom.push_back(t.min_domains > 0 ? t.min_domains : 0);
    // filter: affinity terms, ORed (none when a term is empty: everything matches)
    cp.tg_term_base.push_back((int32_t)cp.tg_terms.size());
    cp.tg_aff.push_back(aff && nonempty ? 1 : 0);
    cp.tg_nterm.push_back(aff && nonempty ? (int32_t)filts.size() : 0);
    if (aff && nonempty)
      for (auto& f : filts) {
        cp.tg_terms.push_back(f);
        cp.tg_terms_negop.push_back(NegOp(d, f));
      }
    cp.tg_filt_tol.push_back(taint ? ltol : ~0ull);
    // NewTopologyGroup: every known domain of the key, with a zero count (ForEachDomain + taint policy)
    uint64_t reg = 0;
    if (k >= 0) {
      const vector<uint64_t>& dm = domains_of(k);
      for (int b = 0; b < 64; b++)
        if (dm[b] && (!taint || (dm[b] & ltol))) reg |= 1ull << b;
    }
    cp.tg_reg.push_back(reg);
    for (int b = 0; b < 64; b++) cp.tg_cnt.push_back(0);
    if (row >= 0) cp.hcnt0.resize((size_t)cp.GH * std::max(E, 1), 0);
    if (cp.track_nodes) {
      cp.tg_reg_static.push_back(reg);
      cp.tg_hrec_total.push_back(0);
      cp.tg_inv_total.push_back(0);
      cp.tg_spread.push_back(1);
      cp.tg_unreg.emplace_back();
    }
    // countDomains: bound pods the selector matches, on nodes the filter admits; then existing nodes' domains
    auto filter_ok = [&](uint32_t ni) {
      const int ts = cp.ex_taintset[ex_pos[ni]];
      if (taint && !((ltol >> ts) & 1)) return false;
      if (!(aff && nonempty)) return true;
      for (auto& f : filts)
        if (HostCompatible(d, node_reqs[ni], f, false)) return true;
      return false;
    };
    const string ns = sh.namespace_ ? sh.namespace_ : "";
    const vector<int>* ords = k >= 0 ? &node_ords(k) : nullptr;  // value ordinal per node (key k's values: word k)
    for (int bi : sets_for(t.selector, ns)) {
      const BoundSet& bs = bsets[bi];
      if (!SelectorMatches(t.selector, bs.labels)) continue;
      for (const uint32_t ni : bs.nodes) {
        if (row >= 0) {  // hostname: the node's label or, failing that, its name — one domain per node
          if (!filter_ok(ni)) continue;
          uint8_t& c = cp.hcnt0[(size_t)row * std::max(E, 1) + ex_pos[ni]];
          if (c < 254) c++;  // (255: an unregistered domain, below)
        } else {
          const int ord = (*ords)[ni];
          if (ord < 0 || !filter_ok(ni)) continue;
          cp.tg_cnt[(size_t)g * 64 + ord]++;
          cp.tg_reg[g] |= 1ull << ord;
          if (cp.track_nodes) cp.node_cnt[ni].push_back(g * 64 + ord);
        }
      }
    }
    if (k >= 0) {  // the existing nodes' domains depend only on (key, node filter): cached across groups
      string fid = key + "|" + std::to_string(aff && nonempty) + fcanon + (taint ? std::to_string(ltol) : string("-"));
      auto it = node_domains.find(fid);
      if (it == node_domains.end()) {
        uint64_t m = 0;
        for (uint32_t ni = 0; ni < in->n_existing; ni++)
          if ((*ords)[ni] >= 0 && filter_ok(ni)) m |= 1ull << (*ords)[ni];
        it = node_domains.emplace(fid, m).first;
      }
      cp.tg_reg[g] |= it->second;
      if (cp.track_nodes)
        for (uint32_t ni = 0; ni < in->n_existing; ni++)
          if ((*ords)[ni] >= 0 && filter_ok(ni)) cp.node_reg[ni].push_back(g * 64 + (*ords)[ni]);
    }
    if (row >= 0 && E && (cp.track_nodes || !live)) {
      // the nodes this group registers: the filter-matching ones with a hostname label, and the nodes of the pods it
      // counted (both uses below)
      const vector<const char*>& hn = node_vals(kHostname);
      vector<char> counted(in->n_existing, 0);
      for (int bi : sets_for(t.selector, ns))
        if (SelectorMatches(t.selector, bsets[bi].labels))
          for (const uint32_t ni : bsets[bi].nodes) counted[ni] = 1;
      // the positions a not-live creation leaves unregistered (below)
      if (cp.track_nodes)
        for (uint32_t ni = 0; ni < in->n_existing; ni++)
          if (!(filter_ok(ni) && (hn[ni] || counted[ni]))) cp.tg_unreg[g].push_back(ex_pos[ni]);
      // a hostname group a relaxation creates (Topology.Update after NewTopology): its domains are only what
      // countDomains registers (NewTopology's Register of every existing node came before it). An unregistered node
      // holds 255: the spread test fails on it until a Record registers it; the NodeClaims created before the group
      // get 255 on the device when the group comes to exist.
      if (!live)
        for (uint32_t ni = 0; ni < in->n_existing; ni++)
          if (!(filter_ok(ni) && (hn[ni] || counted[ni]))) cp.hcnt0[(size_t)row * E + ex_pos[ni]] = 255;
    }
    return g;
  };
  // TopologyTypePodAntiAffinity on the hostname key, as a hostname row whose acceptance test is count == 0 (the
  // pre-pass test count + self <= maxSkew with self = 0, maxSkew = 0); no node filter; identity = (type, key,
  // namespaces, selector). countDomains: bound pods it selects, per node. inverse: a bound pod's own required term
  // (updateInverseAntiAffinity): its counts are the owners' nodes, it constrains the pods it selects, and no
  // placement records into it.
  // the namespaces a term selects (upstream Topology.buildNamespaceList): none given and no namespaceSelector -> the
  // pod's own; else the listed ones plus every cluster namespace whose labels the namespaceSelector matches
  auto nss_of = [&](const kp_pod_affinity_term& t, const char* pod_ns) {
    std::set<string> n;
    for (uint32_t i = 0; i < t.n_namespaces; i++) n.insert(t.namespaces[i] ? t.namespaces[i] : "");
    if (t.has_namespace_selector) {
      for (uint32_t i = 0; i < in->n_namespaces; i++) {
        const kp_namespace& ns = in->namespaces[i];
        std::map<string, string> labels;
        for (uint32_t j = 0; j < ns.n_labels; j++)
          labels[ns.labels[j].key ? ns.labels[j].key : ""] = ns.labels[j].value ? ns.labels[j].value : "";
        if (SelectorMatches(t.namespace_selector, labels)) n.insert(ns.name ? ns.name : "");
      }
    } else if (n.empty()) {
      n.insert(pod_ns ? pod_ns : "");
    }
    return n;
  };
  // TopologyTypePodAffinity (aff): the same hostname row with maxSkew = -1, whose pre-pass test is count > 0, or,
  // while no domain has a count (tg_reg bit 0 clear), the self-selecting pod's bootstrap (nextDomainAffinity).
  // one bound pod counted in group g on input node ni: hostname rows count per node (bit 0 of tg_reg: some domain
  // has a count); dictionary keys count per value ordinal of the node's label (none: not counted)
  auto record_bound = [&](int g, uint32_t ni) {
    if (cp.tg_row[g] >= 0) {
      uint8_t& c = cp.hcnt0[(size_t)cp.tg_row[g] * std::max(E, 1) + ex_pos[ni]];
      if (c < 254) c++;
      cp.tg_reg[g] |= 1;
      if (cp.track_nodes) {
        cp.node_hrec[ni].push_back(g);
        cp.tg_hrec_total[g]++;
      }
    } else {
      const int k = cp.tg_key[g];
      const int ord = node_ords(k)[ni];
      if (ord < 0) return;
      cp.tg_cnt[(size_t)g * 64 + ord]++;
      cp.tg_reg[g] |= 1ull << ord;
      if (cp.track_nodes) cp.node_cnt[ni].push_back(g * 64 + ord);
    }
  };
  auto anti_group = [&](const kp_pod_affinity_term& t, const std::set<string>& nss, bool inverse, bool aff = false) -> int {
    string id = string(inverse ? "inv|" : aff ? "aff|" : "anti|") + (t.topology_key ? t.topology_key : "") + "|";
    for (auto& n : nss) id += n + ",";
    id += "|" + SelectorCanon(t.selector);
    auto it = ids.find(id);
    if (it != ids.end()) return it->second;
    const int g = cp.G++;
    ids[id] = g;
    cp.tg_live.push_back(1);
    g_shape.push_back(-1);
    g_spec.push_back(nullptr);
    g_sel.push_back(&t.selector);
    g_nss.push_back(nss);
    g_inverse.push_back(inverse ? 1 : 0);
    const string key = t.topology_key ? t.topology_key : "";
    int k = -1, row = -1;
    if (key == kHostname) {
      row = cp.GH++;
    } else {  // a dictionary key: counts per value ordinal, registered domains = every known value (no taint policy)
      k = d.key(key);
      if (k < 0) return fail(KP_E_INVAL, "topology key %s missing from the dictionary", key.c_str()), -1;
      if (d.dd.nval[k] > 64) return fail(KP_E_UNSUPPORTED, "topology key %s has > 64 values", key.c_str()), -1;
      if (cp.tkey_slot[k] < 0) {
        cp.tkey_slot[k] = cp.TK++;
        cp.tk_keys.push_back(k);
      }
    }
    cp.tg_key.push_back(k);
    cp.tg_row.push_back(row);
    cp.tg_maxskew.push_back(aff ? -1 : 0);
    cp.tg_mindom.push_back(0);
    cp.tg_term_base.push_back((int32_t)cp.tg_terms.size());
    cp.tg_aff.push_back(0);
    cp.tg_nterm.push_back(0);
    cp.tg_filt_tol.push_back(~0ull);
    uint64_t reg = 0;
    if (cp.track_nodes) {
      cp.tg_reg_static.push_back(0);
      cp.tg_hrec_total.push_back(0);
      cp.tg_inv_total.push_back(0);
      cp.tg_spread.push_back(0);
      cp.tg_unreg.emplace_back();
    }
    if (k >= 0) {
      const vector<uint64_t>& dm = domains_of(k);
      for (int b = 0; b < 64; b++)
        if (dm[b]) reg |= 1ull << b;
      if (cp.track_nodes) cp.tg_reg_static[g] = reg;
      const vector<int>& ords = node_ords(k);
      for (uint32_t ni = 0; ni < in->n_existing; ni++) {
        if (ords[ni] >= 0) {
          reg |= 1ull << ords[ni];
          if (cp.track_nodes) cp.node_reg[ni].push_back(g * 64 + ords[ni]);
        }
      }
    }
    cp.tg_reg.push_back(reg);
    for (int b = 0; b < 64; b++) cp.tg_cnt.push_back(0);
    if (row >= 0) cp.hcnt0.resize((size_t)cp.GH * std::max(E, 1), 0);
    if (!inverse) {  // (the sets of every namespace the term selects, in set order)
      vector<int> sets;
      for (const string& n : nss) {
        const vector<int>& v = sets_for(t.selector, n);
        sets.insert(sets.end(), v.begin(), v.end());
      }
      std::sort(sets.begin(), sets.end());
      for (int bi : sets)
        if (SelectorMatches(t.selector, bsets[bi].labels))
          for (const uint32_t ni : bsets[bi].nodes) record_bound(g, ni);
    }
    return g;
  };
  for (uint32_t p = 0; p < in->n_pods; p++) {  // NewTopology: Update(pod) in pod order
    const uint32_t s = in->pods[p].shape;
    if (seen[s]) continue;
    seen[s] = 1;
    const kp_pod_shape& sh = in->shapes[s];
    for (uint32_t j = 0; j < sh.n_topology_spread; j++) {
      const int g = group_of(s, (int)j, 0, true);
      if (g < 0) return KP_E_UNSUPPORTED;
      sgroup[s].push_back(g);
    }
    for (uint32_t a = 0; a < PodTermCount(sh); a++) {
      bool aff = false;
      const kp_pod_affinity_term& t = *PodTermAt(sh, (int)a, &aff);
      const int g = anti_group(t, nss_of(t, sh.namespace_), false, aff);
      if (g < 0) return KP_E_UNSUPPORTED;
      sgroup[s].push_back(g);
    }
  }
  pt.lap("  topo: NewTopology");
  vector<int> inverse_groups;  // updateInverseAffinities: after the batch's groups
  for (uint32_t b = 0; b < in->n_bound_pods; b++) {
    const kp_bound_pod& bp = in->bound_pods[b];
    for (uint32_t j = 0; j < bp.n_anti_affinity; j++) {
      const kp_pod_affinity_term& t = bp.anti_affinity[j];
      const int g = anti_group(t, nss_of(t, bp.namespace_), true);
      if (g < 0) return KP_E_UNSUPPORTED;
      if (std::find(inverse_groups.begin(), inverse_groups.end(), g) == inverse_groups.end()) inverse_groups.push_back(g);
      record_bound(g, bp.node);
      if (cp.track_nodes) {
        cp.node_inv[bp.node].push_back(g);
        cp.tg_inv_total[g]++;
      }
    }
  }
  // every other group a shape-level owns, before the recording lists are built: the groups of shapes without pods,
  // and the spread groups of relaxed levels (a relaxation makes them exist; records must reach them from then on)
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    const uint32_t n_terms = sh.n_topology_spread + PodTermCount(sh);
    if (sgroup[s].empty() && n_terms) {  // shape without pods: no groups were created for it
      for (uint32_t j = 0; j < sh.n_topology_spread; j++) {
        const int g = group_of(s, (int)j, 0, false);
        if (g < 0) return KP_E_UNSUPPORTED;
        sgroup[s].push_back(g);
      }
      for (uint32_t a = 0; a < PodTermCount(sh); a++) {
        bool aff = false;
        const kp_pod_affinity_term& t = *PodTermAt(sh, (int)a, &aff);
        const int g = anti_group(t, nss_of(t, sh.namespace_), false, aff);
        if (g < 0) return KP_E_UNSUPPORTED;
        sgroup[s].push_back(g);
      }
    }
    for (int l = 1; l < cp.shape_nlevels[s]; l++)
      for (int j : spread_levels[s][l])
        if (j < (int)sh.n_topology_spread && group_of(s, j, l, false) < 0) return KP_E_UNSUPPORTED;
    if (cp.track_nodes)  // sgroup: the level-0 spread groups first, then the pod (anti-)affinity groups
      cp.shape_l0[s].assign(sgroup[s].begin(), sgroup[s].begin() + std::min<size_t>(sgroup[s].size(), sh.n_topology_spread));
  }
  pt.lap("  topo: other groups");
  if (cp.G == 0) return KP_OK;
  if ((size_t)cp.GH * (size_t)(E + in->n_pods) > ((size_t)1 << 31))
    return fail(KP_E_UNSUPPORTED, "%d hostname topologies x %u nodes", cp.GH, E + in->n_pods);
  if (E == 0) cp.hcnt0.clear();
  // recording groups per shape (TopologyGroup.selects: namespace + selector on the pod's labels); shapes are
  // indexed by (namespace, label) so a matchLabels selector only tests the shapes carrying its first label
  vector<std::map<string, string>> shape_labels(in->n_shapes);
  std::map<string, vector<uint32_t>> by_label, by_ns;
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    shape_labels[s] = LabelMap(sh.labels, sh.n_labels);
    const string ns = sh.namespace_ ? sh.namespace_ : "";
    by_ns[ns].push_back(s);
    for (auto& kv : shape_labels[s]) by_label[ns + '\x01' + kv.first + '\x01' + kv.second].push_back(s);
  }
  vector<vector<int>> recs(in->n_shapes);
  static const vector<uint32_t> kNone;
  vector<vector<int>> inv_owned(in->n_shapes);  // inverse groups that select each shape
  for (int g = 0; g < cp.G; g++) {
    const kp_label_selector& sel = *g_sel[g];
    if (sel.is_nil) continue;
    for (const string& ns : g_nss[g]) {
      const vector<uint32_t>* cands;
      if (sel.n_match_labels) {
        auto it = by_label.find(ns + '\x01' + (sel.match_labels[0].key ? sel.match_labels[0].key : "") + '\x01' +
                                (sel.match_labels[0].value ? sel.match_labels[0].value : ""));
        cands = it == by_label.end() ? &kNone : &it->second;
      } else {
        auto it = by_ns.find(ns);
        cands = it == by_ns.end() ? &kNone : &it->second;
      }
      for (uint32_t s : *cands)
        if (SelectorMatches(sel, shape_labels[s])) (g_inverse[g] ? inv_owned[s] : recs[s]).push_back(g);
    }
  }
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    // each group once: the device Record gives every group of a pod its own lane
    std::sort(recs[s].begin(), recs[s].end());
    recs[s].erase(std::unique(recs[s].begin(), recs[s].end()), recs[s].end());
    cp.shape_rec_base[s] = (int32_t)cp.rec_list.size();
    cp.shape_rec_n[s] = (int32_t)recs[s].size();
    cp.rec_list.insert(cp.rec_list.end(), recs[s].begin(), recs[s].end());
  }
  pt.lap("  topo: record lists");
  // owned groups per shape-level: (group, self-selecting, podDomains mask over the key's value ordinals)
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    const uint32_t n_terms = sh.n_topology_spread + PodTermCount(sh);
    if (!n_terms && inv_owned[s].empty()) continue;
    const std::map<string, string> lm = LabelMap(sh.labels, sh.n_labels);
    for (int l = 0; l < cp.shape_nlevels[s]; l++) {
      const int sl = cp.shape_level_base[s] + l;
      vector<int> sp = spread_levels[s][l];  // term ids, then the inverse groups selecting the shape (as -1 - g)
      for (int g : inv_owned[s]) sp.push_back(-1 - g);
      if (sp.size() > 8) return fail(KP_E_UNSUPPORTED, "> 8 topology constraints (spread / anti-affinity) on one pod");
      cp.sl_own_base[sl] = (int32_t)cp.own_group.size();
      cp.sl_own_n[sl] = (int32_t)sp.size();
      const KReqs strict = Compile(d, strict_levels[s][l]);
      for (int j : sp) {
        // spreads: the level's group (a relaxed required term makes another one, live once a pod relaxes to it)
        const int g = j < 0 ? -1 - j : j < (int)sh.n_topology_spread ? group_of(s, j, l, false) : sgroup[s][j];
        if (g < 0) return KP_E_UNSUPPORTED;
        cp.own_group.push_back(g);
        // self: the spread's / affinity term's selector matches the pod (spread: count + 1; affinity: it may
        // bootstrap); anti-affinity accepts count == 0 only
        bool aff = false;
        const kp_pod_affinity_term* pt = j >= (int)sh.n_topology_spread ? PodTermAt(sh, j - (int)sh.n_topology_spread, &aff) : nullptr;
        cp.own_self.push_back(j >= 0 && j < (int)sh.n_topology_spread ? (SelectorMatches(sh.topology_spread[j].selector, lm) ? 1 : 0)
                              : (pt && aff && nss_of(*pt, sh.namespace_).count(sh.namespace_ ? sh.namespace_ : "") &&
                                 SelectorMatches(pt->selector, lm)) ? 1 : 0);
        const int k = cp.tg_key[g];
        uint64_t pd = 0;
        if (k >= 0) {
          for (int b = 0; b < d.dd.nval[k]; b++)
            if (Has(d, strict, k, k * 64 + b)) pd |= 1ull << b;
          cp.sl_topo_keys[sl] |= 1ull << k;
        }
        cp.own_pd.push_back(pd);
        const int32_t rec[8] = {g, cp.own_self.back(), k, cp.tg_maxskew[g], cp.tg_mindom[g], cp.tg_row[g],
                                k >= 0 ? cp.tkey_slot[k] : -1, 0};
        cp.own_rec.insert(cp.own_rec.end(), rec, rec + 8);
      }
    }
  }
  pt.lap("  topo: owned");
  // shape-levels the fast lane may take: at most 4 owned groups, every owned and every recorded group a spread
  // (maxSkew > 0) and no recorded group with node-filter terms (the fast lane's Record reads the NodeClaim's value
  // codes); pods of other levels (affinity, anti-affinity, filtered groups) stay on the full path
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    bool rec_ok = true;
    for (int i = 0; i < cp.shape_rec_n[s]; i++) {
      const int g = cp.rec_list[cp.shape_rec_base[s] + i];
      rec_ok = rec_ok && cp.tg_maxskew[g] > 0 && !cp.tg_aff[g];
    }
    for (int l = 0; l < cp.shape_nlevels[s]; l++) {
      const int sl = cp.shape_level_base[s] + l;
      bool ok = rec_ok && cp.sl_own_n[sl] <= 4;
      for (int j = 0; j < cp.sl_own_n[sl] && ok; j++) ok = cp.tg_maxskew[cp.own_group[cp.sl_own_base[sl] + j]] > 0;
      cp.sl_fast_topo[sl] = ok ? 1 : 0;
    }
  }
  cp.rec_aux.resize(cp.rec_list.size());
  for (size_t i = 0; i < cp.rec_list.size(); i++) {
    const int g = cp.rec_list[i];
    cp.rec_aux[i] = cp.tg_row[g] >= 0 ? cp.tg_row[g] : -1 - cp.tkey_slot[cp.tg_key[g]];
  }
  // existing nodes: value ordinal of each topology key (0xFF: no label)
  cp.ex_tcode.assign((size_t)std::max(cp.TK, 1) * std::max(E, 1), 0xFF);
  for (int k = 0; k < KP_MAX_KEYS; k++) {
    if (cp.tkey_slot[k] < 0) continue;
    const vector<int>& ords = node_ords(k);
    for (int e = 0; e < E; e++)
      if (ords[cp.ex_input[e]] >= 0) cp.ex_tcode[(size_t)cp.tkey_slot[k] * E + e] = (uint8_t)ords[cp.ex_input[e]];
  }
  if (cp.tg_terms.empty()) {
    KReqs z;
    memset(&z, 0, sizeof z);
    cp.tg_terms.push_back(z);
    cp.tg_terms_negop.push_back(0);
  }
  return KP_OK;
}

// An existing node's labels as requirements (NewExistingNode: each label `In {value}`, in input order), without the
// per-label strings of a RawReqs: views into the caller's kp_labels (keys normalized), plus the hostname requirement's
// value when some pod names kubernetes.io/hostname. Thousands of nodes × ~20 labels made the RawReqs form the largest
// part of a Solve's host compile.
struct NodeLabels {
  vector<std::pair<std::string_view, std::string_view>> kv;  // normalized key, value (the hostname label dropped)
  string host;                                               // the hostname requirement's value (has_host)
  bool has_host = false;
};
// karpv1.NormalizedLabels (Normalize) without a string copy: the alias's target or the key itself
std::string_view NormalizeSV(const char* k) {
  static const std::pair<const char*, string> aliases[] = {
      {"failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone"},
      {"beta.kubernetes.io/arch", "kubernetes.io/arch"},
      {"beta.kubernetes.io/os", "kubernetes.io/os"},
      {"beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type"},
      {"failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region"},
      {"topology.ebs.csi.aws.com/zone", "topology.kubernetes.io/zone"},
  };
  for (auto& a : aliases)
    if (strcmp(k, a.first) == 0) return a.second;
  return k;
}
// Dictionary ids of label keys and values by view, memoised per compile (the Dict's maps take strings)
struct LabelIds {
  const Dict& d;
  std::unordered_map<std::string_view, int> key;
  std::unordered_map<int, std::unordered_map<std::string_view, int>> val;
  explicit LabelIds(const Dict& dd) : d(dd) {}
  int k(std::string_view s) {
    auto it = key.find(s);
    if (it != key.end()) return it->second;
    return key.emplace(s, d.key(string(s))).first->second;
  }
  int b(int kk, std::string_view v) {
    auto& m = val[kk];
    auto it = m.find(v);
    if (it != m.end()) return it->second;
    return m.emplace(v, d.bit(kk, string(v))).first->second;
  }
};

// Compile(d, labels as RawReqs) for a NodeLabels: each label Single(In {value}) Added in order, then the hostname one
KReqs CompileNode(const Dict& d, const NodeLabels& nl, LabelIds& ids) {
  KReqs q, s;
  memset(&q, 0, sizeof q);
  memset(&s, 0, sizeof s);
  auto add = [&](int k, int bit) {  // Single(d, {key k, In, {value bit}}) then HostAdd, s back to zero after
    s.present = 1ull << k;
    s.vals[bit / 64] |= 1ull << (bit % 64);
    HostAdd(d, q, s);
    s.vals[bit / 64] = 0;
    s.present = 0;
  };
  for (auto& kv : nl.kv) {
    const int k = ids.k(kv.first);
    add(k, ids.b(k, kv.second));
  }
  if (nl.has_host) {
    const int k = d.key(kHostname);
    add(k, d.bit(k, nl.host));
  }
  return q;
}

// Inputs of one Solve that are not part of its SolveBase: the pods' relaxation levels, node labels, spread keys.
struct SolveRaw {
  vector<RawReqs> np_reqs;                        // per input NodePool (requirements + labels + nodepool key)
  vector<vector<TaintT>> np_taints;
  vector<vector<RawReqs>> levels, strict_levels;  // per shape: NewPodRequirements after successive Relax
  vector<vector<vector<int>>> spread_levels;      // per level: topology terms (j < n_topology_spread: spread j;
                                                  // n_topology_spread + a: anti-affinity term a of AntiTerms)
  vector<vector<vector<RawReqs>>> filter_levels;  // per level: MakeTopologyNodeFilter's terms (nodeSelector + each
                                                  // remaining required term; the nodeSelector alone when none)
  std::set<string> topo_keys;                     // non-hostname spread keys (need a dictionary id)
  bool tolerate_pns = false;                      // some NodePool taint has effect PreferNoSchedule (NewScheduler)
  vector<int> pns_level;                          // per shape: the level toleratePreferNoScheduleTaints adds, or -1
  vector<NodeLabels> ex_labels;                   // per input existing node (hostname: see HostnameValue)
  bool hostname = false;                          // some pod requirement names kubernetes.io/hostname
};

// kubernetes.io/hostname as a requirement key. Upstream gives every NodeClaim `hostname In {a unique placeholder}`
// (NewNodeClaim) and every existing node `hostname In {its hostname}` (NewExistingNode: the label, else the node
// name). A pod's hostname requirement only ever compares those values with the ones it names, so the dictionary
// holds the named values plus two stand-ins: kHostOther for every hostname no pod names, kHostPlaceholder for the
// NodeClaims' (templates carry it; the decoded NodeClaim requirements drop it, as FinalizeScheduling does).
const char* kHostOther = "\x01other-hostname";
const char* kHostPlaceholder = "\x01hostname-placeholder";

void HostnameNames(const kp_requirements& r, bool* used, std::set<string>* named) {
  for (uint32_t i = 0; i < r.n; i++) {
    const kp_requirement& x = r.items[i];
    if (!x.key || string(x.key) != kHostname) continue;
    *used = true;
    for (uint32_t j = 0; j < x.n_values; j++) named->insert(x.values[j] ? x.values[j] : "");
  }
}

void KeyReqs(string& o, const RawReqs& rs) {
  for (auto& r : rs) {
    o += r.key + '\x01' + std::to_string(r.op) + '\x01' + std::to_string(r.minv);
    for (auto& v : r.values) o += '\x02' + v;
    o += '\x03';
  }
  o += '\x04';
}

// The catalogues' seqnums as they are now, and that part of a cache fingerprint.
vector<uint64_t> SeqnumsOf(const vector<const kp_catalog*>& cats) {
  vector<uint64_t> v;
  for (auto* c : cats) v.push_back(c->seqnum);
  return v;
}
// the ctx's cached bases that compiled catalogue c (kp_catalog_destroy)
void DropBasesOf(kp_ctx* ctx, const kp_catalog* c) {
  auto& bases = ctx->bases;
  bases.erase(std::remove_if(bases.begin(), bases.end(),
                             [&](const std::shared_ptr<SolveBase>& b) {
                               return std::find(b->catalogs.begin(), b->catalogs.end(), c) != b->catalogs.end();
                             }),
              bases.end());
}
// KP_OK while every catalogue a base (or plan) compiled is alive, else the error a run or refresh returns.
int32_t CatalogsAlive(const vector<std::shared_ptr<bool>>& alive) {
  for (auto& a : alive)
    if (!*a) return fail(KP_E_INVAL, "a catalogue this plan was prepared on was destroyed (kp_catalog_destroy)");
  return KP_OK;
}
string SeqKey(const vector<uint64_t>& seqs) {
  string k = "#";
  for (uint64_t q : seqs) k += std::to_string(q) + ";";
  return k;
}
// Fingerprint of everything a SolveBase depends on but the seqnums: catalogue identities, the NodePools.
string BaseIdent(const kp_solve_in* in, const SolveRaw& raw) {
  string k;
  for (uint32_t c = 0; c < in->n_catalogs; c++) {
    const kp_catalog* cat = in->catalogs[c];
    k += std::to_string(cat->uid) + ":" + std::to_string(cat->types.size()) + ";";
  }
  for (uint32_t i = 0; i < in->n_nodepools; i++) {
    const kp_nodepool& np = in->nodepools[i];
    k += string(np.name ? np.name : "") + '\x05' + std::to_string(np.weight) + '\x05' + std::to_string(np.catalog);
    KeyReqs(k, raw.np_reqs[i]);
    for (auto& t : raw.np_taints[i]) k += t.key + '\x01' + t.value + '\x01' + std::to_string(t.effect) + '\x02';
    for (int r = 0; r < KP_NRES; r++)
      if ((np.daemon_requests.present >> r) & 1) k += std::to_string(r) + "=" + std::to_string(np.daemon_requests.milli[r]) + ",";
    k += '\x06';
  }
  return k;
}

// Every key / value / bound slot the requirement set needs is already in the dictionary.
bool Covers(const Dict& d, const RawReqs& rs) {
  for (auto& r : rs) {
    const int k = d.key(r.key);
    if (k < 0) return false;
    if ((r.op == KP_OP_GT || r.op == KP_OP_LT || r.minv >= 0) && k >= d.dd.KB) return false;
    if (r.op == KP_OP_IN || r.op == KP_OP_NOT_IN)
      for (auto& v : r.values)
        if (d.bit(k, v) < 0) return false;
  }
  return true;
}
bool BaseCovers(const SolveBase& b, const SolveRaw& raw) {
  for (auto& lv : raw.levels)
    for (auto& r : lv)
      if (!Covers(b.d, r)) return false;
  {  // the node labels: every key and value in the dictionary (In requirements: no bound slots needed)
    LabelIds ids(b.d);
    const int kh = raw.hostname ? b.d.key(kHostname) : -1;
    for (auto& nl : raw.ex_labels) {
      for (auto& kv : nl.kv) {
        const int k = ids.k(kv.first);
        if (k < 0 || ids.b(k, kv.second) < 0) return false;
      }
      if (nl.has_host && (kh < 0 || b.d.bit(kh, nl.host) < 0)) return false;
    }
  }
  for (auto& k : raw.topo_keys)
    if (b.d.key(k) < 0) return false;
  return true;
}

// Parse the NodePools, shapes (relaxation levels) and node labels of a Solve.
int32_t ParseSolve(const kp_solve_in* in, SolveRaw& raw) {
  if (in->n_catalogs == 0 || !in->catalogs) return fail(KP_E_INVAL, "no catalogues");
  for (uint32_t c = 0; c < in->n_catalogs; c++)
    if (!in->catalogs[c]) return fail(KP_E_INVAL, "null catalogue");
  std::set<string> host_named;  // hostname values the pods' requirements name
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    for (uint32_t j = 0; j < sh.n_node_selector; j++)
      if (sh.node_selector[j].key && string(sh.node_selector[j].key) == kHostname) {
        raw.hostname = true;
        host_named.insert(sh.node_selector[j].value ? sh.node_selector[j].value : "");
      }
    for (uint32_t j = 0; j < sh.n_required_terms; j++) HostnameNames(sh.required_terms[j], &raw.hostname, &host_named);
    for (uint32_t j = 0; j < sh.n_preferred_terms; j++) HostnameNames(sh.preferred_terms[j].preference, &raw.hostname, &host_named);
    HostnameNames(kp_requirements{sh.volume_requirements, sh.n_volume_requirements, 0}, &raw.hostname, &host_named);
  }
  raw.np_reqs.resize(in->n_nodepools);
  raw.np_taints.resize(in->n_nodepools);
  for (uint32_t i = 0; i < in->n_nodepools; i++) {
    const kp_nodepool& np = in->nodepools[i];
    if (np.catalog >= in->n_catalogs) return fail(KP_E_INVAL, "nodepool %u: catalogue %u", i, np.catalog);
    RawReqs r = ParseReqs(np.requirements);
    RawReqs l = LabelReqs(np.labels, np.n_labels, false);
    r.insert(r.end(), l.begin(), l.end());
    r.push_back({kNodePool, KP_OP_IN, {np.name ? np.name : ""}, -1});
    for (auto& x : r)
      if (x.key == kHostname) return fail(KP_E_UNSUPPORTED, "hostname requirement on nodepool");
    if (raw.hostname) r.push_back({kHostname, KP_OP_IN, {kHostPlaceholder}, -1});  // NewNodeClaim's placeholder
    raw.np_reqs[i] = std::move(r);
    for (uint32_t j = 0; j < np.n_taints; j++) {
      raw.np_taints[i].push_back({np.taints[j].key ? np.taints[j].key : "", np.taints[j].value ? np.taints[j].value : "",
                                  np.taints[j].effect});
      // upstream NewScheduler: Preferences{ToleratePreferNoSchedule} when any NodePool template taint has that effect
      if (np.taints[j].effect == KP_EFFECT_PREFER_NO_SCHEDULE) raw.tolerate_pns = true;
    }
  }
  raw.pns_level.assign(in->n_shapes, -1);
  raw.levels.assign(in->n_shapes, {});
  raw.strict_levels.assign(in->n_shapes, {});
  raw.spread_levels.assign(in->n_shapes, {});
  raw.filter_levels.assign(in->n_shapes, {});
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    for (uint32_t j = 0; j < sh.n_topology_spread; j++) {
      const kp_topology_spread& t = sh.topology_spread[j];
      const string key = t.topology_key ? t.topology_key : "";
      if (t.max_skew < 1 || t.max_skew > 250) return fail(KP_E_UNSUPPORTED, "topology spread maxSkew %d", t.max_skew);
      if (key != kHostname) raw.topo_keys.insert(key);  // the key gets a dictionary id even if no value names it
    }
    if (sh.n_preferred_terms > 12) return fail(KP_E_UNSUPPORTED, "> 12 preferred terms");
    if (sh.n_preferred_anti_affinity > 12 || sh.n_preferred_affinity > 12)
      return fail(KP_E_UNSUPPORTED, "> 12 preferred pod (anti-)affinity terms");
    for (uint32_t j = 0; j < PodTermCount(sh); j++) {
      const kp_pod_affinity_term& t = *PodTermAt(sh, (int)j);
      const int32_t rc = CheckAntiTerm(t, "shape", s);
      if (rc) return rc;
      if (t.topology_key != string(kHostname)) raw.topo_keys.insert(t.topology_key);
    }
    RawReqs ns = LabelReqs(sh.node_selector, sh.n_node_selector, false);
    vector<RawReqs> req;
    for (uint32_t j = 0; j < sh.n_required_terms; j++) req.push_back(ParseReqs(sh.required_terms[j]));
    if (sh.n_volume_requirements) {  // VolumeTopology.Inject: appended to every required term (one created if none)
      RawReqs v = ParseReqs(kp_requirements{sh.volume_requirements, sh.n_volume_requirements, 0});
      if (req.empty()) req.push_back(v);
      else
        for (auto& t : req) t.insert(t.end(), v.begin(), v.end());
    }
    vector<std::pair<int, RawReqs>> pref;
    for (uint32_t j = 0; j < sh.n_preferred_terms; j++)
      pref.push_back({sh.preferred_terms[j].weight, ParseReqs(sh.preferred_terms[j].preference)});
    auto byw = [](const std::pair<int, RawReqs>& a, const std::pair<int, RawReqs>& b) { return a.first > b.first; };
    std::stable_sort(pref.begin(), pref.end(), byw);  // sort.Slice on <= 12 = insertion sort (stable)
    vector<int> spreads;
    for (uint32_t j = 0; j < sh.n_topology_spread; j++) spreads.push_back((int)j);
    // preferred anti-affinity terms: removePreferredPodAntiAffinityTerm drops the heaviest first (sort.Slice by
    // weight desc on <= 12 terms: insertion sort, stable)
    vector<int> apref, fpref;  // removePreferredPodAffinityTerm, then removePreferredPodAntiAffinityTerm
    for (uint32_t a = 0; a < sh.n_preferred_anti_affinity; a++) apref.push_back((int)a);
    std::stable_sort(apref.begin(), apref.end(), [&](int x, int y) {
      return sh.preferred_anti_affinity[x].weight > sh.preferred_anti_affinity[y].weight;
    });
    for (uint32_t a = 0; a < sh.n_preferred_affinity; a++) fpref.push_back((int)a);
    std::stable_sort(fpref.begin(), fpref.end(), [&](int x, int y) {
      return sh.preferred_affinity[x].weight > sh.preferred_affinity[y].weight;
    });
    const int nS = (int)sh.n_topology_spread, nRA = (int)sh.n_required_anti_affinity,
              nPA = (int)sh.n_preferred_anti_affinity, nRF = (int)sh.n_required_affinity;
    for (;;) {
      RawReqs r = ns;
      if (!pref.empty()) r.insert(r.end(), pref[0].second.begin(), pref[0].second.end());
      if (!req.empty()) r.insert(r.end(), req[0].begin(), req[0].end());
      raw.levels[s].push_back(std::move(r));
      RawReqs strict = ns;  // NewStrictPodRequirements: without the preferred term
      if (!req.empty()) strict.insert(strict.end(), req[0].begin(), req[0].end());
      raw.strict_levels[s].push_back(std::move(strict));
      vector<RawReqs> filt;
      for (auto& t : req) {
        filt.push_back(ns);
        filt.back().insert(filt.back().end(), t.begin(), t.end());
      }
      if (filt.empty()) filt.push_back(ns);
      raw.filter_levels[s].push_back(std::move(filt));
      vector<int> terms = spreads;  // spreads, required anti-affinity terms, remaining preferred ones, affinity alike
      for (int a = 0; a < nRA; a++) terms.push_back(nS + a);
      for (int a : apref) terms.push_back(nS + nRA + a);
      for (int a = 0; a < nRF; a++) terms.push_back(nS + nRA + nPA + a);
      for (int a : fpref) terms.push_back(nS + nRA + nPA + nRF + a);
      raw.spread_levels[s].push_back(terms);
      if (req.size() > 1) {
        req.erase(req.begin());
      } else if (!fpref.empty()) {
        fpref.erase(fpref.begin());
      } else if (!apref.empty()) {
        apref.erase(apref.begin());
      } else if (!pref.empty()) {
        pref.erase(pref.begin());
      } else {  // removeTopologySpreadScheduleAnyway: first ScheduleAnyway constraint, swapped with the last
        size_t i = 0;
        while (i < spreads.size() && sh.topology_spread[spreads[i]].when_unsatisfiable != KP_SCHEDULE_ANYWAY) i++;
        if (i == spreads.size()) break;
        spreads[i] = spreads.back();
        spreads.pop_back();
      }
    }
    // toleratePreferNoScheduleTaints (the last relaxation, only with Preferences.ToleratePreferNoSchedule): appends
    // {Operator: Exists, Effect: PreferNoSchedule} unless a toleration already equals it (corev1 MatchToleration:
    // key, operator, value and effect equal), so the pod's requirements and terms stay those of the last level
    if (raw.tolerate_pns && !HasPnsToleration(sh)) {
      raw.pns_level[s] = (int)raw.levels[s].size();
      raw.levels[s].push_back(raw.levels[s].back());
      raw.strict_levels[s].push_back(raw.strict_levels[s].back());
      raw.filter_levels[s].push_back(raw.filter_levels[s].back());
      raw.spread_levels[s].push_back(raw.spread_levels[s].back());
    }
  }
  PhaseTimer pt;
  for (uint32_t b = 0; b < in->n_bound_pods; b++)  // inverse anti-affinity keys need a dictionary id too
    for (uint32_t j = 0; j < in->bound_pods[b].n_anti_affinity; j++) {
      const char* k = in->bound_pods[b].anti_affinity[j].topology_key;
      if (k && k[0] && string(k) != kHostname) raw.topo_keys.insert(k);
    }
  raw.ex_labels.resize(in->n_existing);
  for (uint32_t i = 0; i < in->n_existing; i++) {
    const kp_existing_node& e = in->existing[i];
    NodeLabels& nl = raw.ex_labels[i];
    nl.kv.reserve(e.n_labels);
    for (uint32_t j = 0; j < e.n_labels; j++) {
      const std::string_view k = NormalizeSV(e.labels[j].key ? e.labels[j].key : "");
      if (k == kHostname) continue;  // (NewExistingNode's hostname requirement, below)
      nl.kv.emplace_back(k, e.labels[j].value ? e.labels[j].value : "");
    }
    if (raw.hostname) {  // NewExistingNode: hostname In {HostName()} (the label, else the node name)
      string host;
      for (uint32_t j = 0; j < e.n_labels; j++)
        if (e.labels[j].key && string(e.labels[j].key) == kHostname && e.labels[j].value) host = e.labels[j].value;
      if (host.empty()) host = e.name ? e.name : "";
      nl.host = host_named.count(host) ? host : string(kHostOther);
      nl.has_host = true;
    }
  }
  pt.lap(" parse: node labels");
  return KP_OK;
}

// Dictionary (catalogues, NodePools + the values `raw` names), catalogue SoA, offering classes, templates.
// The NodeClaimTemplates' InstanceTypeOptions (upstream NewScheduler's pre-filter: the pool's requirements, empty
// requests, a compatible available offering, minValues); pools that keep no type are skipped. Depends on the
// offerings' availability, so an ICE update re-runs it (RefreshOfferings).
void BuildTemplates(const SolveBase& b, vector<int>& tnp, vector<uint64_t>& tX) {
  const Dict& d = b.d;
  const int TW = b.TW;
  tnp.clear();
  tX.clear();
  for (int i : b.np_order) {
    const KReqs& q = b.np_q[i];
    const HostCat& hc = b.cats[b.np_catalog[i]];
    vector<uint64_t> X(TW, 0);
    for (int t = 0; t < hc.T; t++) X[t / 64] |= 1ull << (t % 64);
    int64_t zero[KP_NRES] = {0};
    HostFilterTypes(d, hc, q, TW, zero, X);
    const uint64_t cls = HostAllowedClasses(d, q, b.classes);
    vector<uint64_t> offer(TW, 0);
    for (int c = 0; c < b.C; c++)
      if ((cls >> c) & 1)
        for (int w = 0; w < TW; w++) offer[w] |= hc.offer_avail[(size_t)c * TW + w];
    bool any = false;
    for (int w = 0; w < TW; w++) any |= (X[w] &= offer[w]) != 0;
    if (any && q.hmin) {
      vector<int> ts;
      for (int t = 0; t < hc.T; t++)
        if ((X[t / 64] >> (t % 64)) & 1) ts.push_back(t);
      if (!HostMinValuesOK(d, hc, q, ts)) any = false;
    }
    if (!any) continue;  // "skipping, nodepool requirements filtered out all instance types"
    tnp.push_back(i);
    tX.insert(tX.end(), X.begin(), X.end());
  }
}

int32_t BuildBase(const kp_solve_in* in, const SolveRaw& raw, SolveBase& b) {
  auto t0 = std::chrono::steady_clock::now();
  vector<const kp_catalog*> cats(in->catalogs, in->catalogs + in->n_catalogs);
  DictBuilder db;
  int maxT = 1;
  for (auto* c : cats) {
    maxT = std::max(maxT, (int)c->types.size());
    for (auto& t : c->types) {
      db.addReqs(t.reqs);
      for (auto& o : t.offs) {
        db.addLabel(kCapType, o.ct);
        if (o.has_zone) db.addLabel(kZone, o.zone);
        if (o.has_zid) db.addLabel(kZoneID, o.zid);
        if (o.has_rid) db.addLabel(kResID, o.rid);
        if (o.has_rt) db.addLabel(kResType, o.rt);
      }
    }
  }
  db.bounded[kResID];
  db.bounded[kResType];
  for (auto& r : raw.np_reqs) db.addReqs(r);
  for (auto& lv : raw.levels)
    for (auto& r : lv) db.addReqs(r);
  for (auto& k : raw.topo_keys) db.bounded[k];
  for (auto& nl : raw.ex_labels) {
    for (auto& kv : nl.kv) db.addLabel(string(kv.first), string(kv.second));
    if (nl.has_host) db.addLabel(kHostname, nl.host);
  }
  int32_t rc = db.build(b.d);
  if (rc) return rc;
  const Dict& d = b.d;
  const int TW = (maxT + 63) / 64;
  b.TW = TW;
  b.d.dd.TW = TW;
  b.d.dd.T = maxT;
  // offering classes
  map<ClassKey, int> classes;
  for (auto* c : cats)
    for (auto& t : c->types)
      for (auto& o : t.offs) {
        const ClassKey ck = ClassOf(d, o);
        if (!classes.count(ck)) {
          int id = (int)classes.size();
          classes[ck] = id;
        }
      }
  if (classes.size() > KP_MAX_CLASSES) return fail(KP_E_UNSUPPORTED, "%zu offering classes", classes.size());
  b.C = (int)classes.size();
  b.classes.resize(b.C);
  for (auto& kv : classes) b.classes[kv.second] = ClassOfKey(kv.first);
  b.d.dd.C = b.C;
  b.cats.resize(cats.size());
  uint64_t catalog_keys = 0, multi = 0;
  for (size_t i = 0; i < cats.size(); i++) {
    rc = CompileCatalog(d, cats[i]->types, TW, classes, b.cats[i]);
    if (rc) return rc;
    multi |= b.cats[i].multi_valued;
    for (int k = 0; k < d.dd.K; k++) {
      // NOKEY covers every type only if no type has the key (padding bits masked)
      bool all = true;
      for (int t = 0; t < b.cats[i].T && all; t++)
        if (!((b.cats[i].NOKEY[(size_t)k * TW + t / 64] >> (t % 64)) & 1)) all = false;
      if (!all) catalog_keys |= 1ull << k;
    }
  }
  b.d.dd.catalog_keys = catalog_keys;
  b.d.dd.single_valued = catalog_keys & ~multi;
  for (auto& hc : b.cats) hc.multi_valued = multi;
  // the NodePools' taint sets (ids 0.. in input order; a Solve's nodes add theirs after these)
  map<vector<TaintT>, int> tsets;
  b.np_taintset.resize(in->n_nodepools);
  for (uint32_t i = 0; i < in->n_nodepools; i++) {
    vector<TaintT> v = raw.np_taints[i];
    std::sort(v.begin(), v.end());
    auto it = tsets.find(v);
    if (it == tsets.end()) {
      it = tsets.emplace(v, (int)b.tsets.size()).first;
      b.tsets.push_back(v);
    }
    b.np_taintset[i] = it->second;
  }
  // templates: weight desc, name asc; pre-filter options with empty requests (upstream NewScheduler)
  vector<int> order(in->n_nodepools);
  for (uint32_t i = 0; i < in->n_nodepools; i++) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    const kp_nodepool &p = in->nodepools[x], &q = in->nodepools[y];
    if (p.weight != q.weight) return p.weight > q.weight;
    return strcmp(p.name ? p.name : "", q.name ? q.name : "") < 0;
  });
  b.np_order = order;
  for (uint32_t i = 0; i < in->n_nodepools; i++) {
    const kp_nodepool& np = in->nodepools[i];
    b.np_q.push_back(Compile(d, raw.np_reqs[i]));
    b.np_catalog.push_back((int32_t)np.catalog);
    for (int r = 0; r < KP_NRES; r++)
      b.np_daemon.push_back((np.daemon_requests.present >> r) & 1 ? np.daemon_requests.milli[r] : 0);
  }
  b.catalogs = cats;
  for (auto* c : cats) b.alive.push_back(c->alive);
  b.seqnums = SeqnumsOf(cats);
  rc = ReservationTables(b);
  if (rc) return rc;
  b.d.dd.res_any = b.res_cls ? 1 : 0;
  BuildTemplates(b, b.tmpl_nodepool, b.tmpl_X);
  for (int i : b.tmpl_nodepool) {
    b.tmpl_reqs.push_back(b.np_q[i]);
    b.tmpl_taintset.push_back(b.np_taintset[i]);
    b.tmpl_catalog.push_back(b.np_catalog[i]);
    b.tmpl_daemon.insert(b.tmpl_daemon.end(), b.np_daemon.begin() + (size_t)i * KP_NRES,
                         b.np_daemon.begin() + (size_t)(i + 1) * KP_NRES);
  }
  b.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return KP_OK;
}

// Per-Solve half on a SolveBase: taint sets, limits, existing nodes, shapes (levels, PVP rows), topology, queue.
// Exact Queue keys from the pods' UIDs (upstream NewQueue's last tie-break compares metadata.uid as strings): each
// pod's rank in the batch sorted by UID, equal UIDs (invalid in a cluster) by batch index. false: a NULL UID.
bool ExactUidKeys(const char* const* uids, uint32_t n, vector<uint64_t>& key) {
  // sorted by the first 8 bytes as a big-endian integer (zero-padded: the string order), strcmp only between equal
  // prefixes; equal strings keep their input order
  struct Ent {
    uint64_t pre;
    uint32_t i;
  };
  vector<Ent> e(n);
  for (uint32_t i = 0; i < n; i++) {
    if (!uids[i]) return false;
    uint64_t p = 0;
    const unsigned char* u = (const unsigned char*)uids[i];
    for (int j = 0; j < 8; j++) {
      p = (p << 8) | u[j];
      if (!u[j]) {  // shorter: the rest stays zero
        p <<= 8 * (7 - j);
        break;
      }
    }
    e[i] = {p, i};
  }
  std::sort(e.begin(), e.end(), [&](const Ent& a, const Ent& b) {
    if (a.pre != b.pre) return a.pre < b.pre;
    const int c = strcmp(uids[a.i], uids[b.i]);
    return c != 0 ? c < 0 : a.i < b.i;
  });
  key.assign(n, 0);
  for (uint32_t r = 0; r < n; r++) key[e[r].i] = r;
  return true;
}

int32_t CompilePerCall(const kp_solve_in* in, const SolveRaw& raw, Compiled& cp) {
  const SolveBase& b = *cp.B;
  const Dict& d = b.d;
  const int TW = b.TW;
  PhaseTimer pt;
  map<vector<TaintT>, int> tsets;
  for (size_t i = 0; i < b.tsets.size(); i++) tsets[b.tsets[i]] = (int)i;
  auto tset = [&](vector<TaintT> v) {
    std::sort(v.begin(), v.end());
    auto it = tsets.find(v);
    if (it != tsets.end()) return it->second;
    int id = (int)tsets.size();
    tsets[v] = id;
    return id;
  };
  for (int np : b.tmpl_nodepool) {
    const kp_nodepool& p = in->nodepools[np];
    for (int r = 0; r < KP_NRES; r++) cp.tmpl_remaining.push_back((p.limits.present >> r) & 1 ? p.limits.milli[r] : 0);
    cp.tmpl_limit_present.push_back(p.limits.present);
  }
  // existing nodes: initialized first, then by name
  vector<int> ex(in->n_existing);
  for (uint32_t i = 0; i < in->n_existing; i++) ex[i] = (int)i;
  std::stable_sort(ex.begin(), ex.end(), [&](int x, int y) {
    const kp_existing_node &p = in->existing[x], &q = in->existing[y];
    if ((p.initialized != 0) != (q.initialized != 0)) return p.initialized != 0;
    return strcmp(p.name ? p.name : "", q.name ? q.name : "") < 0;
  });
  LabelIds lids(d);
  for (int i : ex) {
    const kp_existing_node& e = in->existing[i];
    cp.ex_input.push_back(i);
    cp.ex_reqs.push_back(CompileNode(d, raw.ex_labels[i], lids));
    vector<TaintT> ts;
    for (uint32_t j = 0; j < e.n_taints; j++)
      ts.push_back({e.taints[j].key ? e.taints[j].key : "", e.taints[j].value ? e.taints[j].value : "", e.taints[j].effect});
    cp.ex_taintset.push_back(tset(ts));
    for (int r = 0; r < KP_NRES; r++) {
      cp.ex_available.push_back((e.available.present >> r) & 1 ? e.available.milli[r] : 0);
      cp.ex_requests.push_back((e.requests.present >> r) & 1 ? e.requests.milli[r] : 0);
    }
  }
  if (tsets.size() > 64) return fail(KP_E_UNSUPPORTED, "%zu distinct taint sets (max 64)", tsets.size());
  pt.lap(" existing nodes");
  // shapes: levels, negop, tolerations, requests, per-catalogue PVP rows
  int sl = 0;
  for (uint32_t s = 0; s < in->n_shapes; s++) {
    const kp_pod_shape& sh = in->shapes[s];
    cp.shape_level_base.push_back(sl);
    cp.shape_nlevels.push_back((int32_t)raw.levels[s].size());
    for (int r = 0; r < KP_NRES; r++) cp.shape_requests.push_back((sh.requests.present >> r) & 1 ? sh.requests.milli[r] : 0);
    // Taints.ToleratesPod per taint set, with the pod's tolerations (+ toleratePreferNoScheduleTaints' at its level)
    auto tolerates = [&](bool pns) {
      uint64_t tol = 0;
      for (auto& kv : tsets) {
        bool all = true;
        for (auto& taint : kv.first) {
          bool ok = false;
          for (uint32_t j = 0; j < sh.n_tolerations + (pns ? 1 : 0) && !ok; j++) {
            const kp_toleration& t = j < sh.n_tolerations ? sh.tolerations[j] : kPnsToleration;
            const string tk = t.key ? t.key : "", tv = t.value ? t.value : "";
            if (t.effect != KP_EFFECT_ANY && t.effect != taint.effect) continue;
            if (!tk.empty() && tk != taint.key) continue;
            if (t.op == KP_TOL_EQUAL) ok = tv == taint.value;
            else if (t.op == KP_TOL_EXISTS) ok = true;
          }
          if (!ok) all = false;
        }
        if (all) tol |= 1ull << kv.second;
      }
      return tol;
    };
    const uint64_t tol0 = tolerates(false);
    for (size_t l = 0; l < raw.levels[s].size(); l++) {  // per shape-level: the PreferNoSchedule level differs
      const bool pns = (int)l == raw.pns_level[s];
      cp.shape_tolerates.push_back(pns ? tolerates(true) : tol0);
      cp.sl_pns.push_back(pns ? 1 : 0);
    }
    for (auto& lv : raw.levels[s]) {
      KReqs q = Compile(d, lv);
      cp.shape_reqs.push_back(q);
      cp.shape_negop.push_back(NegOp(d, q));
      vector<int32_t> slots(KP_MAX_KEYS, 0);
      for (size_t ci = 0; ci < b.cats.size(); ci++) {
        const HostCat& hc = b.cats[ci];
        cp.pvp_base.push_back((int32_t)(cp.pvp.size() / TW));
        int row = 0;
        if (ci == 0) cp.pvp_n.push_back(0);
        for (int k = 0; k < d.dd.K; k++) {
          if (!((q.present >> k) & 1) || !((d.dd.single_valued >> k) & 1)) continue;
          vector<uint64_t> acc(hc.NOKEY.begin() + (size_t)k * TW, hc.NOKEY.begin() + (size_t)(k + 1) * TW);
          for (int wi = 0, w = kw(d, k, 0); wi < nwords(d, k); wi++, w = wi < nwords(d, k) ? kw(d, k, wi) : 0) {
            uint64_t m = d.dd.validbits[w];
            while (m) {
              int bb = __builtin_ctzll(m);
              m &= m - 1;
              if (Has(d, q, k, w * 64 + bb))
                for (int x = 0; x < TW; x++) acc[x] |= hc.TM[(size_t)(w * 64 + bb) * TW + x];
            }
          }
          cp.pvp.insert(cp.pvp.end(), acc.begin(), acc.end());
          slots[k] = row++;  // same key order for every catalogue -> same relative slot
          if (ci == 0) cp.pvp_n.back() = row;
        }
      }
      cp.pvp_slot.insert(cp.pvp_slot.end(), slots.begin(), slots.end());
      sl++;
    }
  }
  if (cp.pvp.empty()) cp.pvp.assign(TW, 0);
  pt.lap(" shapes");
  {  // host ports: shapes, then the existing nodes in upstream order
    vector<vector<HostPortKey>> hs(in->n_shapes), hn;
    string err;
    for (uint32_t s2 = 0; s2 < in->n_shapes; s2++)
      if (!ParseHostPorts(in->shapes[s2].host_ports, in->shapes[s2].n_host_ports, &hs[s2], &err))
        return fail(KP_E_INVAL, "shape %u: %s", s2, err.c_str());
    for (int i : cp.ex_input) {
      hn.emplace_back();
      if (!ParseHostPorts(in->existing[i].host_ports, in->existing[i].n_host_ports, &hn.back(), &err))
        return fail(KP_E_INVAL, "existing node %d: %s", i, err.c_str());
    }
    const int32_t hrc = EncodeHostPorts(hs, hn, cp);
    if (hrc) return hrc;
  }
  pt.lap(" host ports");
  int32_t rc = CompileTopology(in, cp, raw.strict_levels, raw.spread_levels, b.np_taintset, raw.filter_levels);
  if (rc) return rc;
  pt.lap(" topology");
  // pods: Queue order byCPUAndMemoryDescending (cpu desc, memory desc, creation asc, uid asc)
  cp.pod_shape.resize(in->n_pods);
  cp.queue.resize(in->n_pods);
  for (uint32_t p = 0; p < in->n_pods; p++) {
    if (in->pods[p].shape >= in->n_shapes) return fail(KP_E_INVAL, "pod %u: shape %u", p, in->pods[p].shape);
    cp.pod_shape[p] = (int32_t)in->pods[p].shape;
    cp.queue[p] = (int32_t)p;
  }
  // (cpu desc, memory desc) depends on the shape only: rank the shapes once, then sort the keys themselves
  // (rank, creation, uid, pod) in place, so the comparator reads contiguous memory instead of gathering per pod
  vector<int32_t> sorder(in->n_shapes), srank(in->n_shapes);
  for (uint32_t s2 = 0; s2 < in->n_shapes; s2++) sorder[s2] = (int32_t)s2;
  auto req_of = [&](int s2, int r) { return cp.shape_requests[(size_t)s2 * KP_NRES + r]; };
  std::sort(sorder.begin(), sorder.end(), [&](int x, int y) {
    if (req_of(x, KP_RES_CPU) != req_of(y, KP_RES_CPU)) return req_of(x, KP_RES_CPU) > req_of(y, KP_RES_CPU);
    return req_of(x, KP_RES_MEMORY) > req_of(y, KP_RES_MEMORY);
  });
  for (uint32_t i = 0, r = 0; i < in->n_shapes; i++) {  // equal (cpu, memory) share a rank
    if (i > 0 && (req_of(sorder[i], KP_RES_CPU) != req_of(sorder[i - 1], KP_RES_CPU) ||
                  req_of(sorder[i], KP_RES_MEMORY) != req_of(sorder[i - 1], KP_RES_MEMORY)))
      r = i;
    srank[sorder[i]] = (int32_t)r;
  }
  struct QKey {
    int32_t rank, pod;
    int64_t creation;
    uint64_t uid;
  };
  vector<uint64_t> uidk;  // the UIDs themselves (ABI v10): their rank in string order is the exact key
  if (in->pod_uids && !ExactUidKeys(in->pod_uids, in->n_pods, uidk)) return fail(KP_E_INVAL, "null pod uid");
  pt.lap(" queue: uid ranks");
  // the same order as one sort by (rank, creation, uid, pod): a counting sort by rank (ranks are < n_shapes), then each
  // rank's pods sorted by (creation, uid, pod) — short, cache-resident sorts instead of one over the whole batch
  vector<uint32_t> rstart(in->n_shapes + 1, 0);
  for (uint32_t p = 0; p < in->n_pods; p++) rstart[srank[cp.pod_shape[p]] + 1]++;
  for (uint32_t r = 0; r < in->n_shapes; r++) rstart[r + 1] += rstart[r];
  vector<QKey> qk(in->n_pods);
  {
    vector<uint32_t> fill(rstart.begin(), rstart.end() - 1);
    for (uint32_t p = 0; p < in->n_pods; p++) {
      const int32_t r = srank[cp.pod_shape[p]];
      qk[fill[r]++] = {r, (int32_t)p, in->pods[p].creation_unix, in->pod_uids ? uidk[p] : in->pods[p].uid_key};
    }
  }
  for (uint32_t r = 0; r < in->n_shapes; r++)
    if (rstart[r + 1] - rstart[r] > 1)
      std::sort(qk.begin() + rstart[r], qk.begin() + rstart[r + 1], [](const QKey& p, const QKey& q) {
        if (p.creation != q.creation) return p.creation < q.creation;
        if (p.uid != q.uid) return p.uid < q.uid;
        return p.pod < q.pod;
      });
  for (uint32_t p = 0; p < in->n_pods; p++) cp.queue[p] = qk[p].pod;
  {  // the fast lane's continuation round pays where most queue neighbours share their shape (deployments created in
     // bursts: runs of one shape-level); elsewhere its registers cost more than it saves (measured)
    uint32_t same = 0;
    for (uint32_t p = 1; p < in->n_pods; p++) same += cp.pod_shape[cp.queue[p]] == cp.pod_shape[cp.queue[p - 1]];
    cp.cont_hint = in->n_pods > 1 && 2 * same >= in->n_pods ? 1 : 0;
  }
  pt.lap(" queue");
  return KP_OK;
}

// An ICE update (kp_catalog_update_offerings: availability, prices; never new offering classes) re-applied to a
// SolveBase in place: the offering arrays of every catalogue (FillOfferings with the base's class ids) and the
// templates' options (BuildTemplates), host side, then the same regions of the resident device copy. Returns 0 when
// done (version bumped), 1 when the base must be rebuilt instead (an offering of an unknown class, or the set of
// templates changed: a NodePool whose types all became unavailable, or the reverse), < 0 on a device error.
// Plans prepared on the base before the refresh see it through `version` (kp_solve_run refuses them until
// kp_solve_refresh).
// The refreshed state becomes current (stale checks pass) only here, after every device copy succeeded: a failed
// copy leaves the old seqnums, so the plans stay refused and a retried refresh copies again.
void CommitRefresh(SolveBase& b) {
  b.seqnums = SeqnumsOf(b.catalogs);
  b.key = b.ident + SeqKey(b.seqnums);
  b.version++;
}

int32_t RefreshOfferings(kp_ctx* ctx, SolveBase& b, bool commit = true) {
  map<ClassKey, int> classes;
  for (int c = 0; c < b.C; c++) classes[KeyOfClass(b.classes[c])] = c;
  for (auto* cat : b.catalogs)
    for (auto& t : cat->types)
      for (auto& o : t.offs)
        if (!classes.count(ClassOf(b.d, o))) return 1;
  vector<HostCat> saved;
  for (size_t i = 0; i < b.cats.size(); i++) {
    saved.push_back(HostCat());
    saved.back().offer_avail.swap(b.cats[i].offer_avail);
    saved.back().price.swap(b.cats[i].price);
    saved.back().price_cm.swap(b.cats[i].price_cm);
    saved.back().price_sub.swap(b.cats[i].price_sub);
    FillOfferings(b.d, b.catalogs[i]->types, b.TW, classes, b.cats[i]);
  }
  vector<int> tnp;
  vector<uint64_t> tX;
  BuildTemplates(b, tnp, tX);
  if (tnp != b.tmpl_nodepool) {  // restore: the caller rebuilds a fresh base (other plans may share this one)
    for (size_t i = 0; i < b.cats.size(); i++) {
      b.cats[i].offer_avail.swap(saved[i].offer_avail);
      b.cats[i].price.swap(saved[i].price);
      b.cats[i].price_cm.swap(saved[i].price_cm);
      b.cats[i].price_sub.swap(saved[i].price_sub);
    }
    return 1;
  }
  b.tmpl_X.swap(tX);
  if (ReservationTables(b)) return 1;  // (reservation classes are fixed by the dictionary: cannot fail here)
  if (b.on_device && ctx) {
    uint8_t* base = (uint8_t*)b.dev.p;
    hipStream_t st = ctx->stream;
    for (size_t i = 0; i < b.cats.size(); i++) {
      const HostCat& hc = b.cats[i];
      const CatOffsets& o = b.coffs[i];
      HIPCHK(hipMemcpyAsync(base + o.offer, hc.offer_avail.data(), hc.offer_avail.size() * 8, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(base + o.price, hc.price.data(), hc.price.size() * 8, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(base + o.price_cm, hc.price_cm.data(), hc.price_cm.size() * 8, hipMemcpyHostToDevice, st));
      if (!hc.price_sub.empty())
        HIPCHK(hipMemcpyAsync(base + o.price_sub, hc.price_sub.data(), hc.price_sub.size() * 8, hipMemcpyHostToDevice, st));
    }
    HIPCHK(hipMemcpyAsync(base + b.o_tX, b.tmpl_X.data(), b.tmpl_X.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  if (commit) CommitRefresh(b);
  return 0;
}

// Compile a Solve. With a ctx, the SolveBase comes from (and goes to) the ctx cache when its fingerprint matches
// and its dictionary covers the batch; without one (kp_solve_validate) it is always built.
int32_t CompileSolve(const kp_solve_in* in, Compiled& cp, kp_ctx* cache = nullptr) {
  if (cache) cp.ov = cache->ov;
  SolveRaw raw;
  PhaseTimer pt;
  int32_t rc = ParseSolve(in, raw);
  if (rc) return rc;
  pt.lap("parse");
  const string ident = BaseIdent(in, raw);
  const string key = ident + SeqKey(SeqnumsOf(vector<const kp_catalog*>(in->catalogs, in->catalogs + in->n_catalogs)));
  if (cache) {
    for (int pass = 0; pass < 2; pass++)  // the exact fingerprint; then one whose catalogues only changed seqnum
      for (size_t i = 0; i < cache->bases.size(); i++) {
        auto& b = cache->bases[i];
        if ((pass == 0 ? b->key != key : b->ident != ident) || !BaseCovers(*b, raw)) continue;
        if (pass == 1) {  // an ICE update: re-apply the offerings in place (host + device) instead of a rebuild
          rc = RefreshOfferings(cache, *b);
          if (rc < 0) return rc;
          if (rc > 0) break;  // the templates changed: rebuild
          cp.base_refreshed = true;
        }
        cp.B = b;
        cp.base_hit = true;
        pt.lap("base lookup");
        rc = CompilePerCall(in, raw, cp);
        pt.lap("per-call compile");
        if (rc == KP_OK) {
          std::rotate(cache->bases.begin() + i, cache->bases.begin() + i + 1, cache->bases.end());  // most recent last
          cache->base_hits++;
          return KP_OK;
        }
        if (rc != KP_E_UNSUPPORTED) return rc;
        pass = 2;  // the cached dictionary's extra values may exceed a per-key limit: rebuild for this batch alone
        break;
      }
  }
  Compiled fresh;
  fresh.track_nodes = cp.track_nodes;
  fresh.ov = cp.ov;
  rc = BuildBase(in, raw, *fresh.B);
  if (rc) return rc;
  fresh.B->ident = ident;
  fresh.B->key = key;
  rc = CompilePerCall(in, raw, fresh);
  if (rc) return rc;
  cp = std::move(fresh);
  if (cache) {
    cache->base_misses++;
    for (size_t i = 0; i < cache->bases.size(); i++)
      if (cache->bases[i]->key == key) {
        cache->bases.erase(cache->bases.begin() + i);
        break;
      }
    cache->bases.push_back(cp.B);
    constexpr size_t kMaxBases = 4;
    if (cache->bases.size() > kMaxBases) cache->bases.erase(cache->bases.begin());
  }
  return KP_OK;
}

// Lays out dict + catalogues in `blob`; fills `catoffs` with the device DevCatalog array offset.

void PutCatalogs(Blob& blob, const Compiled& cp, vector<CatOffsets>& offs) {
  for (auto& hc : cp.B->cats) {
    CatOffsets o;
    o.TM = blob.put(hc.TM);
    o.DNE = blob.put(hc.DNE);
    o.NOKEY = blob.put(hc.NOKEY);
    o.alloc = blob.put(hc.alloc);
    o.cap = blob.put(hc.cap);
    o.nonneg = blob.put(hc.nonneg);
    o.fit_vals = blob.put(hc.fit_vals);
    o.fit_n = blob.put(hc.fit_n);
    o.fit_mask = blob.put(hc.fit_mask);
    o.cls = blob.put(cp.B->classes);
    o.offer = blob.put(hc.offer_avail);
    o.price = blob.put(hc.price);
    o.price_cm = blob.put(hc.price_cm);
    o.price_sub = blob.put(hc.price_sub);
    o.rank = blob.put(hc.name_rank);
    o.code = blob.put(hc.code);
    o.multi = blob.put(hc.multi);
    o.custom = blob.put(hc.custom_nonneg);
    offs.push_back(o);
  }
}
vector<DevCatalog> DevCats(uint8_t* base, const Compiled& cp, const vector<CatOffsets>& offs) {
  vector<DevCatalog> out;
  for (size_t i = 0; i < offs.size(); i++) {
    const CatOffsets& o = offs[i];
    DevCatalog c;
    c.TM = (const uint64_t*)(base + o.TM);
    c.DNE = (const uint64_t*)(base + o.DNE);
    c.NOKEY = (const uint64_t*)(base + o.NOKEY);
    c.vint = nullptr;
    c.alloc = (const int64_t*)(base + o.alloc);
    c.cap = (const int64_t*)(base + o.cap);
    c.nonneg = (const uint64_t*)(base + o.nonneg);
    c.fit_vals = (const int64_t*)(base + o.fit_vals);
    c.fit_n = (const int32_t*)(base + o.fit_n);
    c.fit_mask = (const uint64_t*)(base + o.fit_mask);
    c.cls = (const OfferClass*)(base + o.cls);
    c.offer_avail = (const uint64_t*)(base + o.offer);
    c.price = (const double*)(base + o.price);
    c.price_cm = (const double*)(base + o.price_cm);
    c.price_sub = cp.B->cats[i].price_sub.empty() ? nullptr : (const double*)(base + o.price_sub);
    c.name_rank = (const uint32_t*)(base + o.rank);
    c.code = (const uint16_t*)(base + o.code);
    c.multi = (const uint64_t*)(base + o.multi);
    c.custom_nonneg = (const uint64_t*)(base + o.custom);
    c.multi_valued = cp.B->cats[i].multi_valued;
    c.custom_any = cp.B->cats[i].custom_any;
    out.push_back(c);
  }
  return out;
}

// Device layout of one Solve. Offsets are relative to the shared region (the batch's read-only data: shapes, PVP
// rows, topology tables, the template-options table) or to the Solve's arena (its pods, the existing nodes it may
// use, its mutable state, device-only scratch). A single Solve keeps both in one allocation (shared == arena base);
// the batched general-path simulations (GeneralBatch) share one shared region between many arenas.
struct SolveOffs {
  // shared
  size_t slb = 0, snl = 0, sreqs = 0, sneg = 0, sreq = 0, stol = 0, pvp = 0, pvpb = 0, pvps = 0, pvpn = 0, tlp = 0,
         exts = 0, exav = 0, shpc = 0, shpa = 0, tgk = 0, tgr = 0, tgs = 0, tgm = 0, tga = 0, tgtb = 0, tgft = 0,
         tgt = 0, tgtn = 0, tgnt = 0, srb = 0, srn = 0, recl = 0, recx = 0, slft = 0, slob = 0, slon = 0, owng = 0,
         owns = 0, ownp = 0, ownr = 0, sltk = 0, tks = 0, extc = 0, tkk = 0, slsh = 0, tfeas = 0, exul = 0, exuo = 0,
         exui = 0, slst = 0;
  // arena: the Solve's inputs, then its mutable state [mut, mut_end) (restored before every run; [mut, common) is the
  // part a batched simulation patches, [common, mut_end) the part every simulation starts from alike), then
  // device-only regions
  size_t pod_shape = 0, exso = 0, mut = 0, queue = 0, tgc = 0, tglv = 0, tgreg = 0, hcx = 0, common = 0,
         pod_level = 0, lastlen = 0, lastlen_ep = 0, trem = 0, exr = 0, exrq = 0, exroom = 0, exhp = 0, mut_end = 0;
  size_t pristine = 0, ncr = 0, ncX = 0, ncrq = 0, nct = 0, npods = 0, order = 0, chkblk = 0, maxalloc = 0, fitj = 0,
         nchead = 0, nccat = 0, nchp = 0, place = 0, events = 0, stats = 0, ver0 = 0, exver = 0, tver = 0, curnc = 0,
         curex = 0, held = 0, exown = 0, ver_end = 0, fail0 = 0, ncfail = 0, exfail = 0, tfail = 0, chkdead = 0, fail_end = 0,
         opts = 0, nrem = 0, nopt = 0, hcnc = 0, nctc = 0, txl = 0, txlv = 0, slfail = 0, arena_end = 0;
  size_t n_hcnc = 0;
  int ncc = 0, chk_dead_rows = 0, sort_cap = 0, opt_stride = 0;
  bool chk_on = false;
};

// the resources some shape requests or some template's daemon overhead holds: Fits iterates every resource of the
// merged requests
uint32_t RequestedResources(const Compiled& C) {
  uint32_t m = 0;
  for (size_t i = 0; i < C.shape_requests.size(); i++)
    if (C.shape_requests[i] > 0) m |= 1u << (i % KP_NRES);
  for (size_t i = 0; i < C.B->tmpl_daemon.size(); i++)
    if (C.B->tmpl_daemon[i] > 0) m |= 1u << (i % KP_NRES);
  return m;
}

// per existing node: 1 when its unrequested resources never fail a pod (they never change), else 0
vector<uint8_t> ExStatic(const Compiled& C, uint32_t rmask) {
  const int E = (int)C.ex_reqs.size();
  vector<uint8_t> ok(std::max(E, 1), 0);
  for (int e = 0; e < E; e++) {
    bool good = true;
    for (int r = 0; r < KP_NRES; r++) {
      const int64_t av = C.ex_available[(size_t)e * KP_NRES + r], rq = C.ex_requests[(size_t)e * KP_NRES + r];
      if (av < 0 || (!((rmask >> r) & 1) && rq > av)) good = false;
    }
    ok[e] = good ? 1 : 0;
  }
  return ok;
}

// The fast lane's stage record of each shape-level (topology Solves; SolveArgs::sl_stage): everything static the pod
// loop reads at a pod's start in one 256-byte row, so that the next pod's row is one prefetched load (lane d holds
// dword d) instead of three dependent rounds (level -> owned-group base -> owned-group records -> counts).
//   [0] 0: the fast lane may take the level (sl_fast_topo, no host-port conflicts)  [1..2] tolerated taint sets
//   [3] owned groups  [4] 1: no requirements at the level  [5..6] recorded groups: count, rec_list base
//   [8 + 8j ..] owned group j < 4: own_rec's eight dwords  [40 + 2j ..] its podDomains  [48 + 2i ..] recorded
//   group i < 8: (group, rec_aux)
vector<int32_t> StageRecords(const Compiled& C) {
  const size_t SL = C.shape_reqs.size();
  if (!C.G) return vector<int32_t>(64, 0);
  vector<int32_t> st(std::max<size_t>(SL, 1) * 64, 0);
  for (size_t sh = 0; sh < C.shape_level_base.size(); sh++)
    for (int l = 0; l < C.shape_nlevels[sh]; l++) {
      const size_t sl = (size_t)C.shape_level_base[sh] + l;
      int32_t* r = &st[sl * 64];
      r[0] = (1 - C.sl_fast_topo[sl]) + (C.hp_any && C.shape_hp_conf[sh] ? 1 : 0);
      r[1] = (int32_t)(uint32_t)C.shape_tolerates[sl];
      r[2] = (int32_t)(uint32_t)(C.shape_tolerates[sl] >> 32);
      const int on = C.sl_own_n[sl], ob = C.sl_own_base[sl];
      r[3] = on;
      r[4] = C.shape_reqs[sl].present == 0 ? 1 : 0;
      r[5] = C.shape_rec_n[sh];
      r[6] = C.shape_rec_base[sh];
      for (int j = 0; j < std::min(on, 4); j++) {
        for (int k = 0; k < 8; k++) r[8 + 8 * j + k] = C.own_rec[(size_t)(ob + j) * 8 + k];
        r[40 + 2 * j] = (int32_t)(uint32_t)C.own_pd[ob + j];
        r[41 + 2 * j] = (int32_t)(uint32_t)(C.own_pd[ob + j] >> 32);
      }
      for (int i = 0; i < std::min(C.shape_rec_n[sh], 8); i++) {
        r[48 + 2 * i] = C.rec_list[(size_t)C.shape_rec_base[sh] + i];
        r[49 + 2 * i] = C.rec_aux[(size_t)C.shape_rec_base[sh] + i];
      }
    }
  return st;
}

void PutShared(Blob& blob, const Compiled& C, SolveOffs& o) {
  o.slb = blob.put(C.shape_level_base);
  o.snl = blob.put(C.shape_nlevels);
  o.sreqs = blob.put(C.shape_reqs);
  o.sneg = blob.put(C.shape_negop);
  o.sreq = blob.put(C.shape_requests);
  o.stol = blob.put(C.shape_tolerates);
  o.pvp = blob.put(C.pvp);
  o.pvpb = blob.put(C.pvp_base);
  o.pvps = blob.put(C.pvp_slot);
  o.pvpn = blob.put(C.pvp_n);
  o.tlp = blob.put(C.tmpl_limit_present);
  o.exts = blob.put(C.ex_taintset);
  o.exav = blob.put(C.ex_available);
  o.shpc = blob.put(C.shape_hp_conf);
  o.shpa = blob.put(C.shape_hp_add);
  // topology (read-only part)
  o.tgk = blob.put(C.tg_key), o.tgr = blob.put(C.tg_row), o.tgs = blob.put(C.tg_maxskew), o.tgm = blob.put(C.tg_mindom);
  o.tga = blob.put(C.tg_aff), o.tgtb = blob.put(C.tg_term_base), o.tgft = blob.put(C.tg_filt_tol);
  o.tgt = blob.put(C.tg_terms), o.tgtn = blob.put(C.tg_terms_negop), o.tgnt = blob.put(C.tg_nterm);
  o.srb = blob.put(C.shape_rec_base), o.srn = blob.put(C.shape_rec_n), o.recl = blob.put(C.rec_list);
  o.recx = blob.put(C.rec_aux), o.slft = blob.put(C.sl_fast_topo), o.slob = blob.put(C.sl_own_base);
  o.slon = blob.put(C.sl_own_n), o.owng = blob.put(C.own_group), o.owns = blob.put(C.own_self);
  o.ownp = blob.put(C.own_pd), o.ownr = blob.put(C.own_rec), o.sltk = blob.put(C.sl_topo_keys);
  o.tks = blob.put(C.tkey_slot), o.extc = blob.put(C.ex_tcode), o.tkk = blob.put(C.tk_keys);
  // shape of each shape-level (tmpl_feas_kernel)
  vector<int32_t> sl_shape(std::max<size_t>(1, C.shape_reqs.size()), 0);
  for (size_t sh = 0; sh < C.shape_level_base.size(); sh++)
    for (int l = 0; l < C.shape_nlevels[sh]; l++) sl_shape[(size_t)C.shape_level_base[sh] + l] = (int32_t)sh;
  o.slsh = blob.put(sl_shape);
  o.slst = blob.put(StageRecords(C));
}

// The arena's host-initialised part: the pods (pod_shape / queue of Pc entries), the existing nodes' static check,
// then the mutable state.
void PutArena(Blob& blob, const Compiled& C, const vector<int32_t>& pod_shape, const vector<int32_t>& queue, int Pc,
              const vector<uint8_t>& ex_static, uint32_t rmask, SolveOffs& o) {
  const int E = (int)C.ex_reqs.size();
  o.pod_shape = blob.put(pod_shape);
  o.exso = blob.put(ex_static);
  o.mut = blob.reserve(0);
  o.queue = blob.put(queue);
  o.tgc = blob.put(C.tg_cnt);
  o.tglv = blob.put(C.tg_live);
  o.tgreg = blob.put(C.tg_reg);
  o.hcx = blob.put(C.hcnt0);
  o.common = blob.reserve(0);
  const vector<int32_t> zeros_p(Pc, 0);
  o.pod_level = blob.put(zeros_p);
  o.lastlen = blob.put(zeros_p);
  o.lastlen_ep = blob.put(zeros_p);
  o.trem = blob.put(C.tmpl_remaining);
  o.exrq = blob.put(C.ex_requests);
  // headroom rows of the existing nodes for the first four requested resources (req_res_mask order)
  vector<int64_t> ex_room((size_t)4 * std::max(E, 1), INT64_MAX);
  for (int r = 0, k = 0; r < KP_NRES && k < 4; r++) {
    if (!((rmask >> r) & 1)) continue;
    for (int e = 0; e < E; e++)
      ex_room[(size_t)k * E + e] = C.ex_available[(size_t)e * KP_NRES + r] - C.ex_requests[(size_t)e * KP_NRES + r];
    k++;
  }
  o.exroom = blob.put(ex_room);
  o.exhp = blob.put(C.ex_hp);
  // last of the mutable block: a batched simulation does not copy it (copy-on-write from the pristine block, ex_own)
  o.exr = blob.put(C.ex_reqs);
  o.mut_end = blob.host.size();
}

// The arena's device-only regions (after every put of the blob). with_pristine: a device copy of the mutable state
// (single Solves restore from it; batched simulations restore from the shared one).
void ReserveArenaDev(Blob& blob, const Compiled& C, int Pc, int opt_stride, int sort_cap, bool with_pristine, SolveOffs& o,
                     size_t ex_fail_entries = SIZE_MAX) {
  const int TW = C.B->TW, NT = (int)C.B->tmpl_reqs.size(), E = (int)C.ex_reqs.size();
  o.pristine = with_pristine ? blob.reserve_dev(o.mut_end - o.mut) : 0;
  o.ncr = blob.reserve_dev(sizeof(KReqs) * Pc);
  o.ncX = blob.reserve_dev(sizeof(uint64_t) * (size_t)Pc * TW);
  o.ncrq = blob.reserve_dev(sizeof(int64_t) * (size_t)Pc * KP_NRES);
  o.nct = blob.reserve_dev(sizeof(int32_t) * Pc);
  o.npods = blob.reserve_dev(sizeof(int32_t) * Pc);
  o.order = blob.reserve_dev(sizeof(int32_t) * Pc);
  // chunked newNodeClaims order past the LDS sort capacity (blocks + per (shape-level, block) dead marks): only when
  // the Solve can create more NodeClaims than the LDS holds
  o.sort_cap = sort_cap;
  o.chk_on = Pc > sort_cap;
  o.chkblk = blob.reserve_dev(o.chk_on ? sizeof(ChkBlk) * CHK_MAXC : 8);
  o.maxalloc = blob.reserve_dev(sizeof(int64_t) * (size_t)Pc * KP_NRES);
  o.fitj = blob.reserve_dev(sizeof(int32_t) * (size_t)Pc * KP_NRES);
  o.nchead = blob.reserve_dev(sizeof(NcHead) * (size_t)Pc + 64);
  o.nccat = blob.reserve_dev(sizeof(int32_t) * (size_t)Pc);
  o.nchp = blob.reserve_dev(C.hp_any ? sizeof(uint64_t) * (size_t)Pc : 8);
  o.place = blob.reserve_dev(sizeof(int32_t) * Pc);
  o.events = blob.reserve_dev(sizeof(int32_t) * Pc);
  o.stats = blob.reserve_dev(sizeof(uint64_t) * KP_SOLVE_STATS);
  // failure memo (see SolveArgs): versions start at 0, memo entries at -1
  const size_t SLn = std::max<size_t>(1, C.shape_reqs.size());
  o.ncc = (int)std::min<size_t>((size_t)Pc, std::max<size_t>(1, ((size_t)256 << 20) / (4 * SLn)));
  o.ver0 = blob.reserve_dev(0);
  o.exver = blob.reserve_dev(sizeof(int32_t) * std::max(E, 1));
  o.tver = blob.reserve_dev(sizeof(int32_t) * std::max(NT, 1));
  o.curnc = blob.reserve_dev(sizeof(int32_t) * 2 * SLn);  // cursors start at {0, 0} (zeroed per run)
  o.curex = blob.reserve_dev(sizeof(int32_t) * 2 * SLn);
  o.held = blob.reserve_dev(C.B->res_cls ? sizeof(uint64_t) * (size_t)Pc : 8);
  o.exown = blob.reserve_dev(sizeof(uint64_t) * (size_t)std::max(1, (E + 63) / 64));  // copy-on-write bits (zeroed)
  o.ver_end = blob.total();
  o.fail0 = blob.reserve_dev(0);
  o.ncfail = blob.reserve_dev(sizeof(int32_t) * SLn * o.ncc);
  // (batched simulations: one entry per usable-list entry of each shape-level, SolveArgs::ex_ulist)
  o.exfail = blob.reserve_dev(sizeof(int32_t) * (ex_fail_entries != SIZE_MAX ? std::max<size_t>(ex_fail_entries, 1)
                                                                               : SLn * std::max(E, 1)));
  o.tfail = blob.reserve_dev(sizeof(int32_t) * SLn * std::max(NT, 1));
  o.txlv = blob.reserve_dev(sizeof(int32_t) * std::max(NT, 1));  // -1: not computed
  o.slfail = blob.reserve_dev(sizeof(int32_t) * SLn);  // -1: no failure yet
  o.chk_dead_rows = o.chk_on ? (int)std::min<size_t>(SLn, ((size_t)64 << 20) / (4 * CHK_MAXC)) : 0;
  o.chkdead = blob.reserve_dev(std::max<size_t>(sizeof(int32_t) * o.chk_dead_rows * CHK_MAXC, 8));
  o.fail_end = blob.total();
  o.opt_stride = opt_stride;
  o.txl = blob.reserve_dev(sizeof(uint64_t) * (size_t)std::max(NT, 1) * TW);
  o.opts = blob.reserve_dev(sizeof(uint32_t) * (size_t)Pc * opt_stride);
  o.nrem = blob.reserve_dev(sizeof(uint32_t) * Pc);
  o.nopt = blob.reserve_dev(sizeof(uint32_t) * Pc);
  o.n_hcnc = (size_t)C.GH * Pc;
  o.hcnc = blob.reserve_dev(std::max<size_t>(o.n_hcnc, 1));
  o.nctc = blob.reserve_dev(std::max<size_t>((size_t)C.TK * Pc, 1));
  o.arena_end = blob.total();
}

// SolveArgs of one Solve over the shared region `sh` and the arena `ar` (offsets from `o`).
void BindSolve(SolveArgs& a, const Compiled& C, const SolveOffs& o, uint8_t* sh, uint8_t* ar, int n_pods, int Pc,
               uint32_t rmask, int res_mode) {
  uint8_t* cbase = (uint8_t*)C.B->dev.p;
  memset(&a, 0, sizeof a);
  a.dict = (const DevDict*)(cbase + C.B->o_dict);
  a.cats = (const DevCatalog*)(cbase + C.B->o_cats);
  a.n_catalogs = (int32_t)C.B->cats.size();
  a.vint = (const int64_t*)(cbase + C.B->o_vint);
  a.n_pods = n_pods;
  a.pod_shape = (const int32_t*)(ar + o.pod_shape);
  a.pod_level = (int32_t*)(ar + o.pod_level);
  a.queue = (int32_t*)(ar + o.queue);
  a.lastlen = (int32_t*)(ar + o.lastlen);
  a.lastlen_epoch = (int32_t*)(ar + o.lastlen_ep);
  a.shape_level_base = (const int32_t*)(sh + o.slb);
  a.shape_nlevels = (const int32_t*)(sh + o.snl);
  a.shape_reqs = sh + o.sreqs;
  a.shape_negop = (const uint64_t*)(sh + o.sneg);
  a.shape_requests = (const int64_t*)(sh + o.sreq);
  a.shape_tolerates = (const uint64_t*)(sh + o.stol);
  a.shape_pvp = (const uint64_t*)(sh + o.pvp);
  a.pvp_base = (const int32_t*)(sh + o.pvpb);
  a.pvp_slot = (const int32_t*)(sh + o.pvps);
  a.sl_pvp_n = (const int32_t*)(sh + o.pvpn);
  a.n_tmpl = (int32_t)C.B->tmpl_reqs.size();
  a.tmpl_reqs = cbase + C.B->o_treqs;
  a.tmpl_taintset = (const int32_t*)(cbase + C.B->o_tts);
  a.tmpl_catalog = (const int32_t*)(cbase + C.B->o_tcat);
  a.tmpl_X = (const uint64_t*)(cbase + C.B->o_tX);
  a.tmpl_daemon = (const int64_t*)(cbase + C.B->o_tdm);
  a.tmpl_limit_present = (const uint32_t*)(sh + o.tlp);
  a.tmpl_remaining = (int64_t*)(ar + o.trem);
  a.n_existing = (int32_t)C.ex_reqs.size();
  a.ex_reqs = ar + o.exr;
  a.ex_reqs_ro = nullptr;  // (batched simulations: GeneralBatchRun points it at the pristine block)
  a.ex_own = (uint64_t*)(ar + o.exown);
  a.ex_taintset = (const int32_t*)(sh + o.exts);
  a.ex_available = (const int64_t*)(sh + o.exav);
  a.ex_requests = (int64_t*)(ar + o.exrq);
  a.ex_room = (int64_t*)(ar + o.exroom);
  a.nc_reqs = ar + o.ncr;
  a.nc_X = (uint64_t*)(ar + o.ncX);
  a.nc_requests = (int64_t*)(ar + o.ncrq);
  a.nc_tmpl = (int32_t*)(ar + o.nct);
  a.g_npods = (int32_t*)(ar + o.npods);
  a.g_order = (int32_t*)(ar + o.order);
  a.sort_in_lds = 1;
  a.sort_cap = o.sort_cap;
  a.ncc = o.ncc;
  a.chk_blk = (ChkBlk*)(ar + o.chkblk);
  a.chk_dead = (int32_t*)(ar + o.chkdead);
  a.chk_dead_rows = o.chk_dead_rows;
  a.chk_maxc = o.chk_on ? CHK_MAXC : 0;
  if (C.ov.chunk_capacity) a.chk_maxc = o.chk_on ? std::max(0, std::min(CHK_MAXC, C.ov.chunk_capacity)) : 0;
  a.nc_head = (NcHead*)(((uintptr_t)(ar + o.nchead) + 63) & ~(uintptr_t)63);
  a.nc_fail = (int32_t*)(ar + o.ncfail);
  a.ex_ver = (int32_t*)(ar + o.exver);
  a.ex_fail = (int32_t*)(ar + o.exfail);
  a.tmpl_ver = (int32_t*)(ar + o.tver);
  a.tmpl_fail = (int32_t*)(ar + o.tfail);
  a.tmpl_xlim = (uint64_t*)(ar + o.txl);
  a.tmpl_xlim_ver = (int32_t*)(ar + o.txlv);
  a.sl_fail = (int32_t*)(ar + o.slfail);
  a.cur_nc = (int32_t*)(ar + o.curnc);
  a.cur_ex = (int32_t*)(ar + o.curex);
  a.nc_maxalloc = (int64_t*)(ar + o.maxalloc);
  a.nc_fitj = (int32_t*)(ar + o.fitj);
  a.nc_cat = (int32_t*)(ar + o.nccat);
  a.hp_any = C.hp_any ? 1 : 0;
  a.shape_hp_conf = (const uint64_t*)(sh + o.shpc);
  a.shape_hp_add = (const uint64_t*)(sh + o.shpa);
  a.ex_hp = (uint64_t*)(ar + o.exhp);
  a.nc_hp = (uint64_t*)(ar + o.nchp);
  a.req_res_mask = rmask;
  a.n_req_res = __builtin_popcount(rmask);
  a.timing = C.ov.timing ? 1 : 0;
  a.cont = C.ov.fast_lane ? (C.ov.fast_lane == 2 ? 1 : 0) : C.cont_hint;
  a.n_groups = C.G;
  a.tg_key = (const int32_t*)(sh + o.tgk);
  a.tg_row = (const int32_t*)(sh + o.tgr);
  a.tg_maxskew = (const int32_t*)(sh + o.tgs);
  a.tg_mindom = (const int32_t*)(sh + o.tgm);
  a.tg_aff = (const int32_t*)(sh + o.tga);
  a.tg_term_base = (const int32_t*)(sh + o.tgtb);
  a.tg_filt_tol = (const uint64_t*)(sh + o.tgft);
  a.tg_terms = sh + o.tgt;
  a.tg_terms_negop = (const uint64_t*)(sh + o.tgtn);
  a.tg_cnt = (int32_t*)(ar + o.tgc);
  a.tg_live = (int32_t*)(ar + o.tglv);
  a.tg_nterm = (const int32_t*)(sh + o.tgnt);
  a.tg_reg = (uint64_t*)(ar + o.tgreg);
  a.hcnt_ex = ar + o.hcx;
  a.hcnt_nc = ar + o.hcnc;
  a.hnc_stride = Pc;
  a.shape_rec_base = (const int32_t*)(sh + o.srb);
  a.shape_rec_n = (const int32_t*)(sh + o.srn);
  a.rec_list = (const int32_t*)(sh + o.recl);
  a.rec_aux = (const int32_t*)(sh + o.recx);
  a.sl_fast_topo = (const int32_t*)(sh + o.slft);
  a.sl_own_base = (const int32_t*)(sh + o.slob);
  a.sl_own_n = (const int32_t*)(sh + o.slon);
  a.own_group = (const int32_t*)(sh + o.owng);
  a.own_self = (const int32_t*)(sh + o.owns);
  a.own_pd = (const uint64_t*)(sh + o.ownp);
  a.own_rec = (const int4*)(sh + o.ownr);
  a.sl_stage = (const int32_t*)(sh + o.slst);
  a.sl_topo_keys = (const uint64_t*)(sh + o.sltk);
  a.tkey_slot = (const int32_t*)(sh + o.tks);
  a.n_tk = C.TK;
  a.tk_keys = (const int32_t*)(sh + o.tkk);
  a.nc_tcode = ar + o.nctc;
  a.ex_static_ok = ar + o.exso;
  a.ex_tcode = sh + o.extc;
  a.placement = (int32_t*)(ar + o.place);
  a.events = (int32_t*)(ar + o.events);
  a.stats = (uint64_t*)(ar + o.stats);
  a.res_mode = res_mode;
  a.res_cls = C.B->res_cls;
  a.nc_held = (uint64_t*)(ar + o.held);
  for (int c = 0; c < KP_MAX_CLASSES; c++) a.res_cap0[c] = C.B->res_cap0.empty() ? 0 : C.B->res_cap0[c];
}

// The template-options table's launch over rows [row_lo, row_hi) (out: `words` u64 per (shape-level, template)).
TfeasArgs TfeasOf(const SolveArgs& a, const uint8_t* sh, const SolveOffs& o, int rows, int words) {
  TfeasArgs f;
  memset(&f, 0, sizeof f);
  f.dict = a.dict;
  f.cats = a.cats;
  f.n_catalogs = a.n_catalogs;
  f.vint = a.vint;
  f.n_tmpl = a.n_tmpl;
  f.tmpl_reqs = a.tmpl_reqs;
  f.tmpl_catalog = a.tmpl_catalog;
  f.tmpl_X = a.tmpl_X;
  f.tmpl_daemon = a.tmpl_daemon;
  f.shape_reqs = a.shape_reqs;
  f.shape_negop = a.shape_negop;
  f.sl_shape = (const int32_t*)(sh + o.slsh);
  f.shape_requests = a.shape_requests;
  f.shape_pvp = a.shape_pvp;
  f.pvp_base = a.pvp_base;
  f.pvp_slot = a.pvp_slot;
  f.sl_own_n = a.sl_own_n;
  f.req_res_mask = a.req_res_mask;
  f.row_lo = 0;
  f.row_hi = rows;
  f.words = words;
  f.out = (uint64_t*)(sh + o.tfeas);
  return f;
}

// the newNodeClaims order lives in LDS (64 KiB) up to this many NodeClaims, then spills
int SortCapacity(const kp_overrides& ov) { return ov.sort_capacity > 0 ? std::min(8192, ov.sort_capacity) : 8192; }

}  // namespace

extern "C" {

}  // extern "C"

// A communicator of n_ranks kp_ctx (one per GPU): RCCL (kp_comm_init / kp_comm_init_all), or a caller-supplied host
// all-gather (kp_comm_init_host). Its settings are read once here, so that every rank takes the same decisions.
struct kp_comm {
  CtxRef ctx;
  ncclComm_t comm = nullptr;        // RCCL transport (null: host transport)
  kp_allgather_fn host_fn = nullptr;
  void* host_user = nullptr;
  int n_ranks = 1, rank = 0;
  bool no_tfeas = false;            // kp_overrides.template_table at init: no template-options table
  uint64_t tfeas_shard_min = 0;     // shard the table over the ranks from this many (shape-level, template) pairs
  DevBuf buf;  // [0]: this rank's record, [1..n_ranks]: the gathered records
};

namespace {
// All-gather of `bytes` per rank over host buffers (recv: n_ranks * bytes in rank order), through the comm's
// transport. Every rank of a collective step calls this exactly once per step, whatever its local outcome: a rank
// that failed locally sends a record saying so (the callers' status / KP_CHOICE_FAILED records), so no peer is left
// waiting in the collective.
int32_t CommExchange(kp_comm* c, const void* send, void* recv, size_t bytes) {
  if (c->host_fn) {
    if (c->host_fn(c->host_user, c->rank, send, recv, bytes) != 0)
      return fail(KP_E_DEVICE, "host all-gather callback failed (rank %d)", c->rank);
    return KP_OK;
  }
  hipStream_t st = c->ctx->stream;
  if (c->buf.n < bytes * (size_t)(c->n_ranks + 1)) {
    c->buf.reset();
    HIPCHK(c->buf.alloc(bytes * (size_t)(c->n_ranks + 1)));
  }
  uint8_t* dev = (uint8_t*)c->buf.p;
  HIPCHK(hipMemcpyAsync(dev, send, bytes, hipMemcpyHostToDevice, st));
  ncclResult_t r = ncclAllGather(dev, dev + bytes, bytes, ncclUint8, c->comm, st);
  if (r != ncclSuccess) return fail(KP_E_DEVICE, "ncclAllGather: %s", ncclGetErrorString(r));
  HIPCHK(hipMemcpyAsync(recv, dev + bytes, bytes * (size_t)c->n_ranks, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return KP_OK;
}
// Device-to-device all-gather (the template-options table): RCCL directly, or staged through the host transport.
int32_t CommAllGatherDev(kp_comm* c, const void* send, void* recv, size_t bytes) {
  hipStream_t st = c->ctx->stream;
  if (!c->host_fn) {
    ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, c->comm, st);
    if (r != ncclSuccess) return fail(KP_E_DEVICE, "ncclAllGather: %s", ncclGetErrorString(r));
    HIPCHK(hipStreamSynchronize(st));
    return KP_OK;
  }
  vector<uint8_t> hs(bytes), hr(bytes * (size_t)c->n_ranks);
  const hipError_t e = hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, st);
  const hipError_t e2 = e == hipSuccess ? hipStreamSynchronize(st) : e;
  int32_t rc = CommExchange(c, hs.data(), hr.data(), bytes);  // reached even when the copy failed
  if (e2 != hipSuccess) return fail(KP_E_DEVICE, "all-gather staging: %s", hipGetErrorString(e2));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(recv, hr.data(), hr.size(), hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  return KP_OK;
}
void CommReadSettings(kp_comm* c) {
  c->no_tfeas = c->ctx->ov.template_table != 0;
  // the table costs ~10 us per 1k pairs on one GPU and an all-gather tens of us: shard only tables worth it
  c->tfeas_shard_min = 1u << 20;
  if (c->ctx->ov.table_shard_min) c->tfeas_shard_min = c->ctx->ov.table_shard_min;
}
}  // namespace

struct kp_solve_plan {
  CtxRef ctx;
  std::unique_ptr<Compiled> cp;
  DevBuf buf;  // per-Solve arena (the catalogue / template part lives in cp->B->dev, shared through the ctx cache)
  SolveArgs a;
  double catalog_ms = 0;  // SolveBase build time when this prepare missed the cache, else 0
  double compile_ms = 0;  // host CompileSolve time of this prepare (KP_HOST_TIMING)
  size_t o_mut = 0, n_mut = 0, o_pristine = 0, o_ver = 0, n_ver = 0, o_fail = 0, n_fail = 0;
  size_t o_stats = 0, o_npods = 0, o_place = 0, o_events = 0, o_nct = 0, o_ncrq = 0, o_opts = 0, o_nrem = 0,
         o_nopt = 0, o_ncr = 0, o_hcnc = 0, n_hcnc = 0, o_held = 0;
  int opt_stride = 0, P = 0, Pc = 1;
  uint32_t max_types = 0;
  bool any_min = false;
  double prepare_ms = 0;
  uint64_t base_version = 0;  // SolveBase::version the plan's derived data (template-options table) reflects
  TfeasArgs tf;               // the table's launch over every row (kp_solve_refresh recomputes it locally)
  bool tfeas_on = false;
};

extern "C" {

// Compile the batch (dictionary, bitsets, catalogue SoA, templates, shapes, queue order) and upload it:
// after this the whole Solve input is resident in HBM.
// Upload a SolveBase once (dict, parsed integers, catalogue SoA + descriptors, templates); later Solves on the same
// catalogues and NodePools point their kernels at this copy.
static int32_t EnsureBaseOnDevice(kp_ctx* ctx, SolveBase& B) {
  if (B.on_device) return KP_OK;
  Compiled view;
  view.B = std::shared_ptr<SolveBase>(&B, [](SolveBase*) {});  // non-owning: PutCatalogs / DevCats read B
  Blob blob;
  B.o_dict = blob.put(&B.d.dd, 1);
  B.o_vint = blob.put(B.d.vint);
  vector<CatOffsets> coffs;
  PutCatalogs(blob, view, coffs);
  B.coffs = coffs;
  B.o_cats = blob.reserve(sizeof(DevCatalog) * coffs.size());
  B.o_treqs = blob.put(B.tmpl_reqs);
  B.o_tts = blob.put(B.tmpl_taintset);
  B.o_tcat = blob.put(B.tmpl_catalog);
  B.o_tX = blob.put(B.tmpl_X);
  B.o_tdm = blob.put(B.tmpl_daemon);
  HIPCHK(B.dev.alloc(blob.total()));
  uint8_t* base = (uint8_t*)B.dev.p;
  vector<DevCatalog> dc = DevCats(base, view, coffs);
  memcpy(blob.host.data() + B.o_cats, dc.data(), sizeof(DevCatalog) * dc.size());
  HIPCHK(hipMemcpyAsync(base, blob.host.data(), blob.host.size(), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  B.on_device = true;
  return KP_OK;
}

// Compile the batch and upload it. The catalogue half (SolveBase: dictionary, catalogue SoA, templates) is taken
// from the ctx cache when the catalogues (identity + seqnum) and NodePools match and the dictionary covers the
// batch; only the per-Solve half (shapes, existing nodes, topology, queue order) is compiled and uploaded.
static int32_t SolvePrepare(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm, kp_solve_plan** out);
int32_t kp_solve_prepare(kp_ctx* ctx, const kp_solve_in* in, kp_solve_plan** out) {
  return SolvePrepare(ctx, in, nullptr, out);
}
int32_t kp_solve_prepare_comm(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm, kp_solve_plan** out) {
  if (comm && comm->ctx != ctx) return fail(KP_E_INVAL, "communicator belongs to another context");
  return SolvePrepare(ctx, in, comm, out);
}
static int32_t SolvePrepareLocal(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm,
                                 std::unique_ptr<kp_solve_plan>& plan, size_t& gather_chunk, size_t& gather_off);
static int32_t SolvePrepare(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm, kp_solve_plan** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!ctx || !in || !out) return fail(KP_E_INVAL, "null argument");
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  std::unique_ptr<kp_solve_plan> plan;
  size_t chunk = 0, off = 0;
  int32_t rc = SolvePrepareLocal(ctx, in, comm, plan, chunk, off);
  if (comm && comm->n_ranks > 1) {
    // every rank reaches this exchange, failed or not: (status, table chunk bytes) of each rank; the all-gather of
    // the table follows only when every rank prepared and all agree on its size
    const string err = g_err;
    int64_t mine[2] = {rc, (int64_t)chunk};
    vector<int64_t> all(2 * (size_t)comm->n_ranks);
    int32_t xrc = CommExchange(comm, mine, all.data(), sizeof mine);
    if (xrc) return xrc;
    if (rc) {
      g_err = err;
      return rc;
    }
    for (int i = 0; i < comm->n_ranks; i++) {
      if (all[2 * i]) return fail(KP_E_DEVICE, "rank %d failed to prepare the Solve (error %lld)", i, (long long)all[2 * i]);
      if (all[2 * i + 1] != (int64_t)chunk)
        return fail(KP_E_INVAL, "ranks disagree on the template-options table (%lld vs %zu bytes): every rank must "
                    "pass the same batch", (long long)all[2 * i + 1], chunk);
    }
    if (chunk) {
      uint8_t* tab = (uint8_t*)plan->buf.p + off;
      rc = CommAllGatherDev(comm, tab + chunk * comm->rank, tab, chunk);
      if (rc) return rc;
    }
  } else if (rc) {
    return rc;
  }
  plan->prepare_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = plan.release();
  return KP_OK;
}
// Everything of a prepare that involves only this rank: compile, upload, this rank's rows of the template table.
// gather_chunk > 0: the table rows [rank * chunk, (rank + 1) * chunk) bytes at gather_off still need the all-gather.
static int32_t SolvePrepareLocal(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm,
                                 std::unique_ptr<kp_solve_plan>& plan, size_t& gather_chunk, size_t& gather_off) {
  gather_chunk = gather_off = 0;
  HIPCHK(hipSetDevice(ctx->device));
  plan = std::make_unique<kp_solve_plan>();
  plan->ctx = ctx;
  plan->cp = std::make_unique<Compiled>();
  Compiled& C = *plan->cp;
  const auto tc0 = std::chrono::steady_clock::now();
  int32_t rc = CompileSolve(in, C, ctx);
  if (rc) return rc;
  plan->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
  plan->catalog_ms = C.base_hit ? 0 : C.B->build_ms;
  rc = EnsureBaseOnDevice(ctx, *C.B);
  if (rc) return rc;
  const Dict& d = C.B->d;
  const int TW = C.B->TW, P = (int)in->n_pods, NT = (int)C.B->tmpl_reqs.size();
  const int Pc = std::max(P, 1);
  plan->P = P;
  plan->Pc = Pc;
  plan->max_types = in->max_instance_types;
  for (auto& q : C.B->tmpl_reqs) plan->any_min |= q.hmin != 0;
  for (auto& q : C.shape_reqs) plan->any_min |= q.hmin != 0;

  const uint32_t rmask = RequestedResources(C);
  Blob blob;
  SolveOffs o;
  PutShared(blob, C, o);
  PutArena(blob, C, C.pod_shape, C.queue, Pc, ExStatic(C, rmask), rmask, o);
  const size_t host_bytes = blob.host.size();
  const int opt_stride = in->max_instance_types ? (int)in->max_instance_types : std::max(1, d.dd.T);
  ReserveArenaDev(blob, C, Pc, opt_stride, SortCapacity(C.ov), true, o);
  // template options per (shape-level, template): rows split evenly over the communicator's ranks (padded so that
  // every rank contributes the same byte count to the all-gather)
  const int SLi = (int)C.shape_reqs.size();
  const bool tfeas_on = NT > 0 && SLi > 0 && !(comm ? comm->no_tfeas : ctx->ov.template_table != 0);
  // shard the rows over the ranks only when the table is large enough to repay the all-gather (kp_comm settings)
  const bool shard = tfeas_on && comm && comm->n_ranks > 1 && (uint64_t)SLi * NT >= comm->tfeas_shard_min;
  const int n_ranks = shard ? comm->n_ranks : 1, my_rank = shard ? comm->rank : 0;
  const int tf_words = TW + KP_NRES / 2 + 1;
  const int rows_per_rank = (SLi + n_ranks - 1) / n_ranks;
  const size_t tf_bytes = tfeas_on ? (size_t)rows_per_rank * n_ranks * NT * tf_words * sizeof(uint64_t) : 0;
  o.tfeas = blob.reserve_dev(std::max<size_t>(tf_bytes, 8));
  const size_t total_bytes = blob.total();

  // the per-Solve arena: reuse the ctx's spare allocation when it is large enough
  if (ctx->spare && ctx->spare_bytes >= total_bytes) {
    plan->buf.p = ctx->spare;
    plan->buf.n = ctx->spare_bytes;
    ctx->spare = nullptr;
    ctx->spare_bytes = 0;
  } else {
    if (ctx->spare) HIPCHK(hipFree(ctx->spare));
    ctx->spare = nullptr;
    ctx->spare_bytes = 0;
    HIPCHK(plan->buf.alloc(total_bytes));
  }
  uint8_t* base = (uint8_t*)plan->buf.p;
  const size_t n_mut = o.mut_end - o.mut;
  HIPCHK(hipMemcpyAsync(base, blob.host.data(), host_bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(base + o.pristine, base + o.mut, n_mut, hipMemcpyDeviceToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));

  SolveArgs& a = plan->a;
  const int res_mode = !C.B->res_cls ? 0 : in->reserved_offering_mode == KP_RESERVED_STRICT ? 2 : 1;
  BindSolve(a, C, o, base, base, P, Pc, rmask, res_mode);
  plan->o_hcnc = o.hcnc;
  plan->n_hcnc = o.n_hcnc;
  plan->o_held = o.held;
  if (tfeas_on) {  // this rank's rows of the template-options table, then one all-gather (RCCL) of every rank's rows
    plan->tf = TfeasOf(a, base, o, SLi, tf_words);
    plan->tfeas_on = true;
    TfeasArgs f = plan->tf;
    f.row_lo = std::min(SLi, my_rank * rows_per_rank);
    f.row_hi = std::min(SLi, (my_rank + 1) * rows_per_rank);
    HIPCHK(launch_tmpl_feas(f, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (shard) {  // the all-gather of every rank's rows follows in SolvePrepare, after the ranks' status exchange
      gather_chunk = (size_t)rows_per_rank * NT * tf_words * sizeof(uint64_t);
      gather_off = o.tfeas;
    }
    a.tfeas = (const uint64_t*)(base + o.tfeas);
    a.tfeas_words = tf_words;
  }

  plan->o_ver = o.ver0;
  plan->n_ver = o.ver_end - o.ver0;
  plan->o_fail = o.fail0;
  plan->n_fail = o.fail_end - o.fail0;
  plan->o_mut = o.mut;
  plan->n_mut = n_mut;
  plan->o_pristine = o.pristine;
  plan->o_stats = o.stats;
  plan->o_npods = o.npods;
  plan->o_place = o.place;
  plan->o_events = o.events;
  plan->o_nct = o.nct;
  plan->o_ncrq = o.ncrq;
  plan->o_opts = o.opts;
  plan->o_nrem = o.nrem;
  plan->o_nopt = o.nopt;
  plan->o_ncr = o.ncr;
  plan->opt_stride = opt_stride;
  plan->base_version = C.B->version;
  return KP_OK;
}

// kp_solve_run on a plan whose catalogues changed since its data was derived would place pods on stale offerings
static int32_t SolvePlanStale(const kp_solve_plan* plan) {
  const SolveBase& B = *plan->cp->B;
  if (int32_t rc = CatalogsAlive(B.alive)) return rc;
  if (plan->base_version != B.version || SeqnumsOf(B.catalogs) != B.seqnums)
    return fail(KP_E_INVAL, "stale plan: a catalogue's seqnum changed since it was prepared (kp_solve_refresh)");
  return KP_OK;
}

int32_t kp_solve_refresh(kp_solve_plan* plan) {
  if (!plan) return fail(KP_E_INVAL, "null argument");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  SolveBase& B = *plan->cp->B;
  if (int32_t rc = CatalogsAlive(B.alive)) return rc;
  if (SeqnumsOf(B.catalogs) != B.seqnums) {
    int32_t rc = RefreshOfferings(ctx, B);
    if (rc < 0) return rc;
    if (rc > 0)
      return fail(KP_E_INVAL, "the offering update changed which NodePools keep instance types: prepare the Solve again");
  }
  if (plan->base_version != B.version && plan->tfeas_on) {  // the table derives from the templates' options
    HIPCHK(launch_tmpl_feas(plan->tf, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  for (int c = 0; c < KP_MAX_CLASSES; c++) plan->a.res_cap0[c] = B.res_cap0.empty() ? 0 : B.res_cap0[c];
  plan->base_version = B.version;
  return KP_OK;
}

void kp_solve_plan_destroy(kp_solve_plan* p) {
  if (!p) return;
  kp_ctx* ctx = p->ctx;
  {
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    (void)hipSetDevice(ctx->device);
    if (p->buf.p && p->buf.n >= ctx->spare_bytes) {  // keep the larger arena for the next prepare
      if (ctx->spare) (void)hipFree(ctx->spare);
      ctx->spare = p->buf.p;
      ctx->spare_bytes = p->buf.n;
      p->buf.p = nullptr;
      p->buf.n = 0;
    }
  }
  delete p;  // (after the lock: it may drop the context's last reference)
}

// kp_cancel: one int32 flag in pinned, host-mapped memory (written by the host, polled by solve_kernel)
struct kp_cancel {
  CtxRef ctx;
  int32_t* flag = nullptr;  // hipHostMalloc: coherent, mapped; the same address on the device (unified addressing)
};

int32_t kp_cancel_create(kp_ctx* ctx, kp_cancel** out) {
  if (!ctx || !out) return fail(KP_E_INVAL, "null argument");
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  auto c = std::make_unique<kp_cancel>();
  c->ctx = ctx;
  void* p = nullptr;
  HIPCHK(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
  c->flag = (int32_t*)p;
  __atomic_store_n(c->flag, 0, __ATOMIC_SEQ_CST);
  *out = c.release();
  return KP_OK;
}
// lock-free: called from another thread while a run holds the context's lock
int32_t kp_cancel_set(kp_cancel* c) {
  if (!c) return fail(KP_E_INVAL, "null argument");
  __atomic_store_n(c->flag, 1, __ATOMIC_SEQ_CST);
  return KP_OK;
}
int32_t kp_cancel_reset(kp_cancel* c) {
  if (!c) return fail(KP_E_INVAL, "null argument");
  __atomic_store_n(c->flag, 0, __ATOMIC_SEQ_CST);
  return KP_OK;
}
void kp_cancel_destroy(kp_cancel* c) {
  if (!c) return;
  {
    std::lock_guard<std::recursive_mutex> lock(c->ctx->mu);  // (no run is reading it once the lock is ours)
    (void)hipSetDevice(c->ctx->device);
    if (c->flag) (void)hipHostFree(c->flag);
  }
  delete c;
}

// One Solve over resident inputs: restore mutable state, solve_kernel, finalize_kernel, copy results.
int32_t kp_solve_run(kp_solve_plan* plan, kp_solve_result** out) { return kp_solve_run_cancellable(plan, nullptr, out); }

int32_t kp_solve_run_cancellable(kp_solve_plan* plan, kp_cancel* cancel, kp_solve_result** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!plan || !out) return fail(KP_E_INVAL, "null argument");
  if (cancel && cancel->ctx.p != plan->ctx.p) return fail(KP_E_INVAL, "the cancel token belongs to another context");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  if (int32_t rc = SolvePlanStale(plan)) return rc;
  HIPCHK(hipSetDevice(ctx->device));
  // (a token already set: nothing is queued on the stream)
  if (cancel && __atomic_load_n(cancel->flag, __ATOMIC_SEQ_CST)) return fail(KP_E_CANCELED, "cancelled before the run");
  const Compiled& C = *plan->cp;
  const Dict& d = C.B->d;
  uint8_t* base = (uint8_t*)plan->buf.p;
  const int P = plan->P, Pc = plan->Pc, opt_stride = plan->opt_stride;
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(base + plan->o_mut, base + plan->o_pristine, plan->n_mut, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemsetAsync(base + plan->o_stats, 0, sizeof(uint64_t) * KP_SOLVE_STATS, st));
  HIPCHK(hipMemsetAsync(base + plan->o_npods, 0, sizeof(int32_t) * Pc, st));
  HIPCHK(hipMemsetAsync(base + plan->o_place, 0xFF, sizeof(int32_t) * Pc, st));
  HIPCHK(hipMemsetAsync(base + plan->o_ver, 0, plan->n_ver, st));
  HIPCHK(hipMemsetAsync(base + plan->o_fail, 0xFF, plan->n_fail, st));
  if (plan->n_hcnc) HIPCHK(hipMemsetAsync(base + plan->o_hcnc, 0, plan->n_hcnc, st));
  SolveArgs a = plan->a;
  if (cancel) {
    void* dp = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dp, cancel->flag, 0));
    a.cancel = (const int32_t*)dp;
  }
  const size_t dyn = std::max<size_t>((size_t)2 * a.sort_cap * sizeof(int32_t), a.chk_maxc ? CHK_LDS_BYTES : 0);
  HIPCHK(hipEventRecord(ctx->ev0, st));
  HIPCHK(launch_solve(a, 8, dyn, st));
  HIPCHK(hipEventRecord(ctx->ev1, st));
  uint64_t stats[KP_SOLVE_STATS];
  HIPCHK(hipMemcpyAsync(stats, base + plan->o_stats, sizeof stats, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (stats[7]) return fail(KP_E_DEVICE, "solve_kernel exceeded its Queue.Pop bound (%llu pops): aborted",
                            (unsigned long long)stats[2]);
  if (stats[46]) return fail(KP_E_CANCELED, "Solve cancelled after %llu pops (kp_cancel_set)", (unsigned long long)stats[2]);
  const int n_nc = (int)stats[3];
  FinalizeArgs f;
  f.solve_stats = nullptr;
  f.dict = a.dict;
  f.cats = a.cats;
  f.vint = a.vint;
  f.n_nc = n_nc;
  f.nc_tmpl = a.nc_tmpl;
  f.tmpl_catalog = a.tmpl_catalog;
  f.nc_reqs = a.nc_reqs;
  f.nc_X = a.nc_X;
  f.max_types = (int32_t)plan->max_types;
  f.opt_stride = opt_stride;
  f.out_options = (uint32_t*)(base + plan->o_opts);
  f.out_n_remaining = (uint32_t*)(base + plan->o_nrem);
  f.out_n_options = (uint32_t*)(base + plan->o_nopt);
  f.nc_held = a.res_mode ? a.nc_held : nullptr;
  HIPCHK(hipEventRecord(ctx->ev2, st));
  HIPCHK(launch_finalize(f, st));
  HIPCHK(hipEventRecord(ctx->ev3, st));

  auto res = std::make_unique<kp_solve_result>();
  res->placement.assign(P, -1);
  const int nn = std::max(n_nc, 1);
  vector<int32_t> place(Pc), events(Pc), nct(nn);
  vector<int64_t> ncrq((size_t)nn * KP_NRES);
  vector<uint32_t> opts((size_t)nn * opt_stride), nrem(nn), nopt(nn);
  HIPCHK(hipMemcpyAsync(place.data(), base + plan->o_place, sizeof(int32_t) * Pc, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(events.data(), base + plan->o_events, sizeof(int32_t) * Pc, hipMemcpyDeviceToHost, st));
  if (n_nc) {
    HIPCHK(hipMemcpyAsync(nct.data(), base + plan->o_nct, sizeof(int32_t) * n_nc, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(ncrq.data(), base + plan->o_ncrq, sizeof(int64_t) * n_nc * KP_NRES, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(opts.data(), base + plan->o_opts, sizeof(uint32_t) * (size_t)n_nc * opt_stride,
                          hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(nrem.data(), base + plan->o_nrem, sizeof(uint32_t) * n_nc, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(nopt.data(), base + plan->o_nopt, sizeof(uint32_t) * n_nc, hipMemcpyDeviceToHost, st));
  }
  vector<KReqs> fin;
  vector<uint64_t> held;
  if (n_nc) {
    fin.resize(n_nc);
    HIPCHK(hipMemcpyAsync(fin.data(), base + plan->o_ncr, sizeof(KReqs) * n_nc, hipMemcpyDeviceToHost, st));
    if (a.res_mode) {
      held.resize(n_nc);
      HIPCHK(hipMemcpyAsync(held.data(), base + plan->o_held, sizeof(uint64_t) * n_nc, hipMemcpyDeviceToHost, st));
    }
  }
  HIPCHK(hipStreamSynchronize(st));
  // FinalizeScheduling: a NodeClaim holding reservations launches only into them (reservation-id In {held ids}; the
  // held classes are compatible with its requirements, so the intersection is exactly that set)
  for (int i = 0; i < (int)held.size(); i++) {
    if (!held[i]) continue;
    const int k = d.key(kResID);
    KReqs& q = fin[i];
    for (int wi = 0; wi < nwords(d, k); wi++) q.vals[kw(d, k, wi)] = 0;
    for (uint64_t m = held[i]; m; m &= m - 1) {
      const int bit = C.B->classes[__builtin_ctzll(m)].rid_bit;
      q.vals[bit / 64] |= 1ull << (bit % 64);
    }
    q.present |= 1ull << k;
    q.compl_ &= ~(1ull << k);
  }
  float ms_solve = 0, ms_fin = 0;
  HIPCHK(hipEventElapsedTime(&ms_solve, ctx->ev0, ctx->ev1));
  HIPCHK(hipEventElapsedTime(&ms_fin, ctx->ev2, ctx->ev3));

  res->ncs.resize(n_nc);
  const int n_ev = (int)stats[4];
  for (int i = 0; i < n_ev; i++) {
    const int p = events[i];
    const int t = place[p];
    if (t >= 0) {
      res->ncs[t].pods.push_back((uint32_t)p);
      res->placement[p] = t;
    } else if (t <= -2) {
      res->placement[p] = -2 - C.ex_input[-2 - t];
    }
  }
  res->fin = fin;
  res->nc_cat.resize(n_nc);
  for (int i = 0; i < n_nc; i++) {
    auto& nc = res->ncs[i];
    res->nc_cat[i] = C.B->tmpl_catalog[nct[i]];
    nc.nodepool = (uint32_t)C.B->tmpl_nodepool[nct[i]];
    nc.n_remaining = nrem[i];
    memset(&nc.requests, 0, sizeof nc.requests);
    for (int r = 0; r < KP_NRES; r++) {
      nc.requests.milli[r] = ncrq[(size_t)i * KP_NRES + r];
      if (nc.requests.milli[r]) nc.requests.present |= 1u << r;
    }
    nc.options.assign(opts.begin() + (size_t)i * opt_stride, opts.begin() + (size_t)i * opt_stride + nopt[i]);
    nc.reqs = DecodeReqs(d, fin[i]);
    // Truncate(reqs, max): minValues must still hold on the truncated options, else the pods fail
    if (!fin.empty() && (fin[i].hmin & fin[i].present)) {
      const HostCat& hc = C.B->cats[C.B->tmpl_catalog[nct[i]]];
      vector<int> ts(nc.options.begin(), nc.options.end());
      if (!HostMinValuesOK(d, hc, fin[i], ts)) {
        for (uint32_t p : nc.pods) res->placement[p] = -1;
        nc.options.clear();
      }
    }
  }
  memset(&res->stats, 0, sizeof res->stats);
  res->stats.device_ms = ms_solve + ms_fin;
  res->stats.solve_kernel_ms = ms_solve;
  res->stats.finalize_kernel_ms = ms_fin;
  res->stats.attempts = stats[0];
  res->stats.bytes_algorithmic = stats[1];
  res->stats.pops = stats[2];
  res->stats.prepare_ms = plan->prepare_ms;
  res->stats.catalog_ms = plan->catalog_ms;
  res->stats.catalog_cached = plan->cp->base_hit ? 1 : 0;
  res->stats.catalog_refreshed = plan->cp->base_refreshed ? 1 : 0;
  for (int i = 0; i < 8; i++) res->stats.phase_cycles[i] = stats[8 + i];
  res->stats.scanned = stats[5];
  res->stats.cursor_starts = stats[6];
  for (int i = 0; i < 8; i++) res->stats.attempt_cycles[i] = stats[16 + i];
  res->stats.fast_pods = stats[24];
  res->stats.slow_sorts = stats[31];
  for (int i = 0; i < 6; i++) res->stats.fast_cycles[i] = stats[25 + i];
  for (int i = 0; i < 8; i++) res->stats.fast_bails[i] = stats[32 + i];
  res->stats.reserved_offering_errors = stats[40];
  for (int i = 0; i < 5; i++) res->stats.order_chunks[i] = stats[41 + i];
  res->stats.run_length_pods = stats[47];
  res->stats.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = res.release();
  return KP_OK;
}

// Host half of kp_solve_prepare without a device: the Go shim's "can the device path take this batch" probe.
int32_t kp_solve_validate(const kp_solve_in* in) {
  if (!in) return fail(KP_E_INVAL, "null argument");
  Compiled C;
  return CompileSolve(in, C);
}

int32_t kp_solve(kp_ctx* ctx, const kp_solve_in* in, kp_solve_result** out) { return kp_solve_cancellable(ctx, in, nullptr, out); }

int32_t kp_solve_cancellable(kp_ctx* ctx, const kp_solve_in* in, kp_cancel* cancel, kp_solve_result** out) {
  kp_solve_plan* plan = nullptr;
  int32_t rc = kp_solve_prepare(ctx, in, &plan);
  if (rc) return rc;
  rc = kp_solve_run_cancellable(plan, cancel, out);
  kp_solve_plan_destroy(plan);
  return rc;
}

uint32_t kp_result_nodeclaim_count(const kp_solve_result* r) { return r ? (uint32_t)r->ncs.size() : 0; }
int32_t kp_result_pod_placements(const kp_solve_result* r, int32_t* out, uint32_t n) {
  if (!r || !out || n != r->placement.size()) return fail(KP_E_INVAL, "bad placement buffer");
  memcpy(out, r->placement.data(), sizeof(int32_t) * n);
  return KP_OK;
}
int32_t kp_result_nodeclaim(const kp_solve_result* r, uint32_t i, kp_nodeclaim_info* out) {
  if (!r || !out || i >= r->ncs.size()) return fail(KP_E_INVAL, "bad nodeclaim index");
  const auto& n = r->ncs[i];
  out->nodepool = n.nodepool;
  out->n_pods = (uint32_t)n.pods.size();
  out->n_remaining = n.n_remaining;
  out->n_options = (uint32_t)n.options.size();
  out->pods = n.pods.data();
  out->options = n.options.data();
  out->requests = n.requests;
  out->requirements.items = n.reqs ? n.reqs->items.data() : nullptr;
  out->requirements.n = n.reqs ? (uint32_t)n.reqs->items.size() : 0;
  out->requirements.reserved_ = 0;
  return KP_OK;
}
int32_t kp_result_stats(const kp_solve_result* r, kp_solve_stats* out) {
  if (!r || !out) return fail(KP_E_INVAL, "null");
  *out = r->stats;
  return KP_OK;
}
void kp_result_destroy(kp_solve_result* r) { delete r; }

// CompatibleAvailableFilter batched on the GPU.
}  // extern "C"

namespace {
// Dictionary + catalogue SoA for a batch of query rows against ONE catalogue (CompatibleAvailableFilter rows,
// launch requests): the catalogue's labels and offerings plus the rows' requirements, compiled rows in qreqs.
int32_t CompileQueries(const kp_catalog* cat, const vector<RawReqs>& qs, Compiled& cp, vector<KReqs>& qreqs) {
  DictBuilder db;
  for (auto& t : cat->types) {
    db.addReqs(t.reqs);
    for (auto& o : t.offs) {
      db.addLabel(kCapType, o.ct);
      db.addLabel(kZone, o.zone);
      if (o.has_zid) db.addLabel(kZoneID, o.zid);
      if (o.has_rid) db.addLabel(kResID, o.rid);
      if (o.has_rt) db.addLabel(kResType, o.rt);
    }
  }
  db.bounded[kResID];
  db.bounded[kResType];
  for (auto& q : qs) db.addReqs(q);
  int32_t rc = db.build(cp.B->d);
  if (rc) return rc;
  const int T = (int)cat->types.size(), TW = std::max(1, (T + 63) / 64);
  cp.B->d.dd.T = T;
  cp.B->d.dd.TW = TW;
  cp.B->TW = TW;  // FillOfferings (kp_*_refresh) lays the offering masks out with it
  map<ClassKey, int> classes;
  const Dict& d = cp.B->d;
  for (auto& t : cat->types)
    for (auto& o : t.offs) {
      const ClassKey ck = ClassOf(d, o);
      if (!classes.count(ck)) {
        int id = (int)classes.size();
        classes[ck] = id;
      }
    }
  if (classes.size() > KP_MAX_CLASSES) return fail(KP_E_UNSUPPORTED, "%zu offering classes", classes.size());
  cp.B->C = (int)classes.size();
  cp.B->d.dd.C = cp.B->C;
  cp.B->classes.resize(cp.B->C);
  for (auto& kv : classes) cp.B->classes[kv.second] = ClassOfKey(kv.first);
  cp.B->cats.resize(1);
  rc = CompileCatalog(d, cat->types, TW, classes, cp.B->cats[0]);
  if (rc) return rc;
  uint64_t catalog_keys = 0;
  for (int k = 0; k < d.dd.K; k++)
    for (int t = 0; t < T; t++)
      if (!((cp.B->cats[0].NOKEY[(size_t)k * TW + t / 64] >> (t % 64)) & 1)) catalog_keys |= 1ull << k;
  cp.B->d.dd.catalog_keys = catalog_keys;
  cp.B->d.dd.single_valued = catalog_keys & ~cp.B->cats[0].multi_valued;
  qreqs.assign(std::max<size_t>(qs.size(), 1), KReqs{});
  for (size_t i = 0; i < qs.size(); i++) qreqs[i] = Compile(d, qs[i]);
  return KP_OK;
}

}  // namespace

// Shared by kp_filter_refresh / kp_launch_refresh: rebuild the offering section of a plan's compiled catalogue
// from the catalogue's current offerings (class ids as compiled) and copy it over the resident arrays.
static int32_t RefreshOfferings(kp_ctx* ctx, const kp_catalog* cat, Compiled& cp, const CatOffsets& coff, uint8_t* base) {
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  map<ClassKey, int> classes;
  for (int c = 0; c < cp.B->C; c++) classes[KeyOfClass(cp.B->classes[c])] = c;
  HostCat hc;  // filled aside: the plan's host copy changes only once the device copy did
  hc.T = cp.B->cats[0].T;
  hc.S = cp.B->cats[0].S;
  try {
    FillOfferings(cp.B->d, cat->types, cp.B->TW, classes, hc);
  } catch (const std::out_of_range&) {
    return fail(KP_E_INVAL, "refresh: an offering outside the plan's offering classes");
  }
  HIPCHK(hipMemcpyAsync(base + coff.offer, hc.offer_avail.data(), hc.offer_avail.size() * sizeof(uint64_t),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(base + coff.price, hc.price.data(), hc.price.size() * sizeof(double),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(base + coff.price_cm, hc.price_cm.data(), hc.price_cm.size() * sizeof(double),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(base + coff.price_sub, hc.price_sub.data(), hc.price_sub.size() * sizeof(double),
                        hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  HostCat& dst = cp.B->cats[0];
  dst.offer_avail.swap(hc.offer_avail);
  dst.price.swap(hc.price);
  dst.price_cm.swap(hc.price_cm);
  dst.price_sub.swap(hc.price_sub);
  return KP_OK;
}

struct kp_filter_plan {
  CtxRef ctx;
  DevBuf buf;
  FeasArgs fa;
  uint32_t n_queries = 0;
  int T = 0;
  size_t tiles = 0, o_mask = 0, o_ch = 0, o_cls = 0;
  bool compact = false;  // KP_FILTER_COMPACT: classes per row instead of the cheapest-price rows
  int ch_stride = 0;  // doubles per device cheapest-price row (whole 128-byte lines; the caller's rows are T long)
  bool cheapest = false;
  double prepare_ms = 0;
  const kp_catalog* cat = nullptr;  // kp_filter_refresh: catalogue, compiled form and its offering offsets
  std::shared_ptr<bool> alive;      // cat's alive token: run / refresh after kp_catalog_destroy return KP_E_INVAL
  uint64_t seqnum = 0;              // catalogue seqnum the resident offerings reflect
  Compiled cp;
  CatOffsets coff{};
};

extern "C" {

// Compile the query rows against the catalogue dictionary and upload rows + catalogue SoA (resident).
int32_t kp_filter_prepare(kp_ctx* ctx, const kp_catalog* cat, const kp_feasibility_query* queries, uint32_t n_queries,
                          int32_t with_cheapest, kp_filter_plan** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!ctx || !cat || (!queries && n_queries) || !out) return fail(KP_E_INVAL, "null argument");
  if (with_cheapest < KP_FILTER_MASK_ONLY || with_cheapest > KP_FILTER_COMPACT)
    return fail(KP_E_INVAL, "with_cheapest %d", with_cheapest);
  const bool compact = with_cheapest == KP_FILTER_COMPACT;
  if (compact) with_cheapest = 0;  // (no price rows: the classes and the resident class prices instead)
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  auto plan = std::make_unique<kp_filter_plan>();
  plan->ctx = ctx;
  plan->compact = compact;
  Compiled cp;
  vector<RawReqs> qs(n_queries);
  for (uint32_t i = 0; i < n_queries; i++) qs[i] = ParseReqs(queries[i].requirements);
  vector<KReqs> qreqs;
  int32_t rc = CompileQueries(cat, qs, cp, qreqs);
  if (rc) return rc;
  const int T = (int)cat->types.size();
  vector<int64_t> qrq((size_t)std::max<uint32_t>(n_queries, 1) * KP_NRES, 0);
  for (uint32_t i = 0; i < n_queries; i++)
    for (int r = 0; r < KP_NRES; r++)
      qrq[(size_t)i * KP_NRES + r] = (queries[i].requests.present >> r) & 1 ? queries[i].requests.milli[r] : 0;
  Blob blob;
  const size_t o_dict = blob.put(&cp.B->d.dd, 1);
  const size_t o_vint = blob.put(cp.B->d.vint);
  vector<CatOffsets> coffs;
  PutCatalogs(blob, cp, coffs);
  const size_t o_cats = blob.reserve(sizeof(DevCatalog));
  const size_t o_q = blob.put(qreqs);
  const size_t o_qr = blob.put(qrq);
  const size_t host_bytes = blob.host.size();
  const size_t tiles = (size_t)(T + 63) / 64;
  plan->o_mask = blob.reserve(sizeof(uint64_t) * std::max<size_t>(1, n_queries * tiles));
  plan->ch_stride = (T + 15) & ~15;
  plan->o_ch = with_cheapest ? blob.reserve(sizeof(double) * std::max<size_t>(1, (size_t)n_queries * plan->ch_stride)) : 0;
  plan->o_cls = compact ? blob.reserve(sizeof(uint64_t) * std::max<size_t>(1, n_queries)) : 0;
  HIPCHK(hipMalloc(&plan->buf.p, blob.host.size()));
  uint8_t* base = (uint8_t*)plan->buf.p;
  vector<DevCatalog> dc = DevCats(base, cp, coffs);
  memcpy(blob.host.data() + o_cats, dc.data(), sizeof(DevCatalog));
  HIPCHK(hipMemcpyAsync(base, blob.host.data(), host_bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  FeasArgs& fa = plan->fa;
  fa.dict = (const DevDict*)(base + o_dict);
  fa.cat = (const DevCatalog*)(base + o_cats);
  fa.vint = (const int64_t*)(base + o_vint);
  fa.T = T;
  fa.n_queries = (int32_t)n_queries;
  fa.mode_compatible = 1;
  fa.pad_ = 0;
  fa.q_reqs = base + o_q;
  fa.q_requests = (const int64_t*)(base + o_qr);
  fa.out_mask = (uint64_t*)(base + plan->o_mask);
  fa.out_cheapest = with_cheapest ? (double*)(base + plan->o_ch) : nullptr;
  fa.out_classes = compact ? (uint64_t*)(base + plan->o_cls) : nullptr;
  fa.ch_stride = plan->ch_stride;
  // the bitset kernel (KP_FEAS_GLOBAL: the per-type global-gather kernel, kept as its cross-check)
  const kp_overrides& ov = plan->ctx->ov;
  fa.bits = ov.feasibility_kernel == 1 ? 0 : 1;
  fa.blocks = (int32_t)std::min<uint32_t>(std::max<uint32_t>((n_queries + 7) / 8, 1), 8192);
  if (ov.feasibility_blocks > 0) fa.blocks = std::min(65535, ov.feasibility_blocks);  // measurement knob
  fa.pad_ = ov.feasibility_temporal ? 0 : 1;  // bit 0: the cheapest-price stream as non-temporal stores
  fa.one_row = ov.feasibility_kernel == 2 ? 1 : 0;  // cross-check: the one-row-per-wave kernel at any catalogue size
  plan->n_queries = n_queries;
  plan->T = T;
  plan->tiles = tiles;
  plan->cheapest = with_cheapest != 0;
  plan->cat = cat;
  plan->alive = cat->alive;
  plan->seqnum = cat->seqnum;
  plan->coff = coffs[0];
  plan->cp = std::move(cp);
  plan->prepare_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = plan.release();
  return KP_OK;
}

// One launch over the resident rows. Results are copied out only into the non-NULL buffers.
int32_t kp_filter_run(kp_filter_plan* plan, uint64_t* out_mask, double* out_cheapest, kp_solve_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!plan) return fail(KP_E_INVAL, "null argument");
  if (out_cheapest && !plan->cheapest) return fail(KP_E_INVAL, "plan was prepared without cheapest prices");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  if (int32_t rc = CatalogsAlive({plan->alive})) return rc;
  if (plan->cat->seqnum != plan->seqnum)  // R:instancetype.go:225-237: a changed seqnum invalidates the offerings
    return fail(KP_E_INVAL, "stale plan: catalogue seqnum %llu, plan built at %llu (kp_filter_refresh)",
                (unsigned long long)plan->cat->seqnum, (unsigned long long)plan->seqnum);
  HIPCHK(hipSetDevice(ctx->device));
  uint8_t* base = (uint8_t*)plan->buf.p;
  const uint32_t n = plan->n_queries;
  HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
  if (n) HIPCHK(launch_feasibility(plan->fa, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
  if (n && out_mask)
    HIPCHK(hipMemcpyAsync(out_mask, base + plan->o_mask, sizeof(uint64_t) * n * plan->tiles, hipMemcpyDeviceToHost, ctx->stream));
  if (n && out_cheapest)
    HIPCHK(hipMemcpy2DAsync(out_cheapest, sizeof(double) * plan->T, base + plan->o_ch, sizeof(double) * plan->ch_stride,
                            sizeof(double) * plan->T, n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->device_ms = ms;
    stats->attempts = (uint64_t)n * plan->T;  // (row, type) pairs evaluated
    stats->prepare_ms = plan->prepare_ms;
    stats->host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return KP_OK;
}

// The compact result: the same launch, the rows' class sets copied out instead of the price rows.
int32_t kp_filter_run_compact(kp_filter_plan* plan, uint64_t* out_mask, uint64_t* out_classes, kp_solve_stats* stats) {
  if (!plan) return fail(KP_E_INVAL, "null argument");
  if (out_classes && !plan->compact) return fail(KP_E_INVAL, "plan was not prepared with KP_FILTER_COMPACT");
  int32_t rc = kp_filter_run(plan, out_mask, nullptr, stats);
  if (rc || !out_classes || !plan->n_queries) return rc;
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(out_classes, (uint8_t*)plan->buf.p + plan->o_cls, sizeof(uint64_t) * plan->n_queries,
                        hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return KP_OK;
}

// The per-(class, type) cheapest available offering prices the compact result indexes (class-major, +inf: none),
// as the plan's resident catalogue holds them (kp_filter_refresh keeps them current).
int32_t kp_filter_class_prices(kp_filter_plan* plan, double* out, uint32_t capacity, uint32_t* n_classes) {
  if (!plan || !n_classes) return fail(KP_E_INVAL, "null argument");
  std::lock_guard<std::recursive_mutex> lock(plan->ctx->mu);
  if (int32_t rc = CatalogsAlive({plan->alive})) return rc;
  if (plan->cat->seqnum != plan->seqnum)  // (a consumer caches the table per seqnum: never hand out the old prices)
    return fail(KP_E_INVAL, "stale plan: catalogue seqnum %llu, plan built at %llu (kp_filter_refresh)",
                (unsigned long long)plan->cat->seqnum, (unsigned long long)plan->seqnum);
  const HostCat& hc = plan->cp.B->cats[0];
  const int C = plan->cp.B->C, T = plan->T;
  *n_classes = (uint32_t)C;
  if (!out) return KP_OK;
  if ((size_t)capacity < (size_t)C * T) return fail(KP_E_INVAL, "capacity %u < %d classes x %d types", capacity, C, T);
  for (int c = 0; c < C; c++)
    for (int t = 0; t < T; t++) out[(size_t)c * T + t] = hc.price_cm[(size_t)c * hc.S + t];
  return KP_OK;
}

// ICE refresh of a prepared plan: FillOfferings over the catalogue's current offerings with the plan's own class
// ids, then only the offering arrays are copied over their resident copies.
int32_t kp_filter_refresh(kp_filter_plan* plan, const kp_catalog* cat) {
  if (!plan || !cat) return fail(KP_E_INVAL, "null argument");
  if (int32_t rc = CatalogsAlive({plan->alive})) return rc;
  if (cat != plan->cat || (int)cat->types.size() != plan->T)
    return fail(KP_E_INVAL, "kp_filter_refresh: the plan was prepared on another catalogue");
  const int32_t rc = RefreshOfferings(plan->ctx, cat, plan->cp, plan->coff, (uint8_t*)plan->buf.p);
  if (rc == KP_OK) plan->seqnum = cat->seqnum;
  return rc;
}

void kp_filter_plan_destroy(kp_filter_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  delete p;
}

int32_t kp_filter_compatible_available(kp_ctx* ctx, const kp_catalog* cat, const kp_feasibility_query* queries,
                                       uint32_t n_queries, uint64_t* out_mask, double* out_cheapest,
                                       kp_solve_stats* stats) {
  if (!out_mask) return fail(KP_E_INVAL, "null argument");
  kp_filter_plan* plan = nullptr;
  int32_t rc = kp_filter_prepare(ctx, cat, queries, n_queries, out_cheapest != nullptr, &plan);
  if (rc) return rc;
  rc = kp_filter_run(plan, out_mask, out_cheapest, stats);
  kp_filter_plan_destroy(plan);
  return rc;
}

// ---- launch-side selection (instance.DefaultProvider.Create), batched over NodeClaims -----------------
}  // extern "C"

// Launch-side reservation tables per (type, class): the cheapest offering at any availability (CapacityBlockFilter
// reads unavailable offerings too, R:filter.go:177-189) and the greatest ReservationCapacity over the available
// offerings (ReservedOfferingFilter, R:filter.go:247-251).
static void FillReservationTables(const Dict& d, const vector<HostType>& types, const map<ClassKey, int>& cls_id, int C,
                                  vector<double>& price_all, vector<int32_t>& rcap) {
  const size_t T = types.size();
  price_all.assign(std::max<size_t>(T * C, 1), std::numeric_limits<double>::infinity());
  rcap.assign(std::max<size_t>(T * C, 1), INT32_MIN);
  for (size_t t = 0; t < T; t++)
    for (auto& o : types[t].offs) {
      const int c = cls_id.at(ClassOf(d, o));
      double& p = price_all[t * C + c];
      if (o.price < p) p = o.price;
      if (o.available) rcap[t * C + c] = std::max(rcap[t * C + c], o.rcap);
    }
}

struct kp_launch_plan {
  CtxRef ctx;
  DevBuf buf;
  LaunchArgs la;
  uint32_t n = 0, max_types = 0, ovr_stride = 0;
  size_t o_out = 0, o_types = 0, o_ovr = 0, o_stats = 0, o_pall = 0, o_rcap = 0;
  double prepare_ms = 0;
  const kp_catalog* cat = nullptr;  // kp_launch_refresh
  std::shared_ptr<bool> alive;      // cat's alive token (as kp_filter_plan)
  uint64_t seqnum = 0;              // catalogue seqnum the resident offerings reflect
  int T = 0;
  Compiled cp;
  CatOffsets coff{};
};
static_assert(sizeof(LaunchOut) == sizeof(kp_launch_result), "LaunchOut mirrors kp_launch_result");

extern "C" {

int32_t kp_launch_prepare(kp_ctx* ctx, const kp_catalog* cat, const kp_launch_request* reqs, uint32_t n,
                          const char* const* subnet_zones, uint32_t n_subnet_zones, uint32_t max_types,
                          kp_launch_plan** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!ctx || !cat || (!reqs && n) || !out || (!subnet_zones && n_subnet_zones)) return fail(KP_E_INVAL, "null argument");
  if (max_types == 0 || max_types > LAUNCH_CAP) return fail(KP_E_INVAL, "max_types %u not in [1, %d]", max_types, LAUNCH_CAP);
  if (n_subnet_zones > 255) return fail(KP_E_UNSUPPORTED, "%u subnet zones", n_subnet_zones);
  const int T = (int)cat->types.size();
  for (auto& t : cat->types) {
    // overrides per type <= subnet zones: one offering per (capacity type, zone), except reserved ones, which the
    // ReservedOfferingFilter narrows to one per zone (then one per (zone, reservation) keeps classes single)
    std::set<std::tuple<string, string, string, string>> seen;
    for (auto& o : t.offs) {
      const bool res = o.ct == "reserved";
      if (o.has_zone && !seen.insert({o.ct, o.zone, res ? o.rid : "", res ? o.rt : ""}).second)
        return fail(KP_E_UNSUPPORTED, "%s: two %s offerings in zone %s", t.name.c_str(), o.ct.c_str(), o.zone.c_str());
    }
  }
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  auto plan = std::make_unique<kp_launch_plan>();
  plan->ctx = ctx;
  Compiled cp;
  vector<RawReqs> qs(n);
  vector<uint32_t> off(n + 1, 0), list;
  for (uint32_t i = 0; i < n; i++) {
    qs[i] = ParseReqs(reqs[i].requirements);
    if (reqs[i].n_instance_types > LAUNCH_CAP)
      return fail(KP_E_UNSUPPORTED, "request %u: %u instance types", i, reqs[i].n_instance_types);
    if (reqs[i].n_instance_types && !reqs[i].instance_types) return fail(KP_E_INVAL, "request %u: null list", i);
    for (uint32_t j = 0; j < reqs[i].n_instance_types; j++) {
      if (reqs[i].instance_types[j] >= (uint32_t)T) return fail(KP_E_INVAL, "request %u: type %u", i, reqs[i].instance_types[j]);
      list.push_back(reqs[i].instance_types[j]);
    }
    off[i + 1] = (uint32_t)list.size();
  }
  if (T > 4096) return fail(KP_E_UNSUPPORTED, "%d instance types", T);
  vector<KReqs> qreqs;
  int32_t rc = CompileQueries(cat, qs, cp, qreqs);
  if (rc) return rc;
  const Dict& d = cp.B->d;
  const int TW = cp.B->d.dd.TW, C = cp.B->C;
  vector<int64_t> qrq((size_t)std::max<uint32_t>(n, 1) * KP_NRES, 0);
  for (uint32_t i = 0; i < n; i++)
    for (int r = 0; r < KP_NRES; r++)
      qrq[(size_t)i * KP_NRES + r] = (reqs[i].requests.present >> r) & 1 ? reqs[i].requests.milli[r] : 0;
  // ExoticInstanceTypeFilter's predicate (R:filter.go:295-310): a metal size or accelerator capacity
  vector<uint64_t> exotic(TW, 0);
  const string kSize = "karpenter.k8s.aws/instance-size";
  for (int t = 0; t < T; t++) {
    const HostType& ht = cat->types[t];
    bool exo = false;
    for (auto& r : ht.reqs)
      if (r.key == kSize && r.op == KP_OP_IN)
        for (auto& v : r.values)
          if (v.find("metal") != string::npos) exo = true;
    for (int r : {KP_RES_NEURON, KP_RES_NEURONCORE, KP_RES_AMD_GPU, KP_RES_NVIDIA_GPU, KP_RES_GAUDI})
      if (((ht.cap_present >> r) & 1) && ht.cap[r] != 0) exo = true;
    if (exo) exotic[t / 64] |= 1ull << (t % 64);
  }
  // offering classes in each type's offering order; class -> subnet zone; capacity-type class masks
  int MO = 1;
  for (auto& t : cat->types) MO = std::max(MO, (int)t.offs.size() + 1);
  vector<uint8_t> ofs_cls((size_t)T * MO, 0xFF);
  const int kct = d.key(kCapType), kz = d.key(kZone);
  std::map<ClassKey, int> cls_id;
  for (int c = 0; c < C; c++) cls_id[KeyOfClass(cp.B->classes[c])] = c;
  for (int t = 0; t < T; t++) {
    int j = 0;
    for (auto& o : cat->types[t].offs) ofs_cls[(size_t)t * MO + j++] = (uint8_t)cls_id.at(ClassOf(d, o));
  }
  const int spot_bit = kct >= 0 ? d.bit(kct, "spot") : -1, od_bit = kct >= 0 ? d.bit(kct, "on-demand") : -1;
  const int res_bit = kct >= 0 ? d.bit(kct, "reserved") : -1, krt = d.key(kResType);
  const int rt0_bit = krt >= 0 ? d.bit(krt, "default") : -1, rt1_bit = krt >= 0 ? d.bit(krt, "capacity-block") : -1;
  uint64_t cls_res = 0, cls_rt0 = 0, cls_rt1 = 0;
  for (int c = 0; c < C; c++) {
    const OfferClass& oc = cp.B->classes[c];
    if (res_bit >= 0 && oc.ct_bit == res_bit) cls_res |= 1ull << c;
    if (rt0_bit >= 0 && oc.rt_bit == rt0_bit) cls_rt0 |= 1ull << c;
    if (rt1_bit >= 0 && oc.rt_bit == rt1_bit) cls_rt1 |= 1ull << c;
  }
  vector<double> price_all;
  vector<int32_t> rcap;
  FillReservationTables(d, cat->types, cls_id, C, price_all, rcap);
  uint64_t cls_spot = 0, cls_od = 0;
  vector<int8_t> cls_zone(std::max(C, 1), -1);
  for (int c = 0; c < C; c++) {
    if (spot_bit >= 0 && cp.B->classes[c].ct_bit == spot_bit) cls_spot |= 1ull << c;
    if (od_bit >= 0 && cp.B->classes[c].ct_bit == od_bit) cls_od |= 1ull << c;
    for (uint32_t z = 0; z < n_subnet_zones; z++)
      if (kz >= 0 && cp.B->classes[c].zone_bit >= 0 && subnet_zones[z] && d.bit(kz, subnet_zones[z]) == cp.B->classes[c].zone_bit) {
        cls_zone[c] = (int8_t)z;
        break;
      }
  }
  Blob blob;
  const size_t o_dict = blob.put(&cp.B->d.dd, 1);
  const size_t o_vint = blob.put(cp.B->d.vint);
  vector<CatOffsets> coffs;
  PutCatalogs(blob, cp, coffs);
  const size_t o_cats = blob.reserve(sizeof(DevCatalog));
  const size_t o_q = blob.put(qreqs);
  const size_t o_qr = blob.put(qrq);
  const size_t o_off = blob.put(off);
  if (list.empty()) list.push_back(0);
  const size_t o_list = blob.put(list);
  const size_t o_exo = blob.put(exotic);
  const size_t o_cz = blob.put(cls_zone);
  const size_t o_oc = blob.put(ofs_cls);
  plan->o_pall = blob.put(price_all);
  plan->o_rcap = blob.put(rcap);
  const size_t host_bytes = blob.host.size();
  const uint32_t ovr_stride = std::max<uint32_t>(1, max_types * std::max<uint32_t>(1, n_subnet_zones));
  plan->o_out = blob.reserve(sizeof(kp_launch_result) * std::max<uint32_t>(n, 1));
  plan->o_types = blob.reserve(sizeof(uint32_t) * (size_t)std::max<uint32_t>(n, 1) * max_types);
  plan->o_ovr = blob.reserve(sizeof(uint32_t) * (size_t)std::max<uint32_t>(n, 1) * ovr_stride);
  plan->o_stats = blob.reserve(sizeof(uint64_t) * 2);
  HIPCHK(hipMalloc(&plan->buf.p, blob.host.size()));
  uint8_t* base = (uint8_t*)plan->buf.p;
  vector<DevCatalog> dc = DevCats(base, cp, coffs);
  memcpy(blob.host.data() + o_cats, dc.data(), sizeof(DevCatalog));
  HIPCHK(hipMemcpyAsync(base, blob.host.data(), host_bytes, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  LaunchArgs& la = plan->la;
  memset(&la, 0, sizeof la);
  la.dict = (const DevDict*)(base + o_dict);
  la.cat = (const DevCatalog*)(base + o_cats);
  la.vint = (const int64_t*)(base + o_vint);
  la.n = (int32_t)n;
  la.max_types = (int32_t)max_types;
  la.spot_bit = spot_bit;
  la.od_bit = od_bit;
  la.ct_key = kct;
  la.MO = MO;
  la.cls_spot = cls_spot;
  la.cls_od = cls_od;
  la.res_bit = res_bit;
  la.cls_res = cls_res;
  la.cls_rt0 = cls_rt0;
  la.cls_rt1 = cls_rt1;
  la.price_all = (const double*)(base + plan->o_pall);
  la.rcap = (const int32_t*)(base + plan->o_rcap);
  la.q_reqs = base + o_q;
  la.q_requests = (const int64_t*)(base + o_qr);
  la.list_off = (const uint32_t*)(base + o_off);
  la.list = (const uint32_t*)(base + o_list);
  la.exotic = (const uint64_t*)(base + o_exo);
  la.cls_zone = (const int8_t*)(base + o_cz);
  la.ofs_cls = base + o_oc;
  la.ovr_stride = ovr_stride;
  la.out = (LaunchOut*)(base + plan->o_out);
  la.out_types = (uint32_t*)(base + plan->o_types);
  la.out_overrides = (uint32_t*)(base + plan->o_ovr);
  la.stats = (uint64_t*)(base + plan->o_stats);
  plan->n = n;
  plan->max_types = max_types;
  plan->ovr_stride = ovr_stride;
  plan->cat = cat;
  plan->alive = cat->alive;
  plan->seqnum = cat->seqnum;
  plan->T = T;
  plan->coff = coffs[0];
  plan->cp = std::move(cp);
  plan->prepare_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = plan.release();
  return KP_OK;
}

// One launch over the resident requests; results copied only into the non-NULL buffers (out_types:
// [n][max_types], out_overrides: [n][max_types * n_subnet_zones]).
int32_t kp_launch_run(kp_launch_plan* plan, kp_launch_result* out, uint32_t* out_types, uint32_t* out_overrides,
                      kp_solve_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!plan) return fail(KP_E_INVAL, "null argument");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  if (int32_t rc = CatalogsAlive({plan->alive})) return rc;
  if (plan->cat->seqnum != plan->seqnum)
    return fail(KP_E_INVAL, "stale plan: catalogue seqnum %llu, plan built at %llu (kp_launch_refresh)",
                (unsigned long long)plan->cat->seqnum, (unsigned long long)plan->seqnum);
  HIPCHK(hipSetDevice(ctx->device));
  uint8_t* base = (uint8_t*)plan->buf.p;
  const uint32_t n = plan->n;
  HIPCHK(hipMemsetAsync(base + plan->o_stats, 0, sizeof(uint64_t) * 2, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
  if (n) HIPCHK(launch_launch(plan->la, ctx->stream));
  HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
  uint64_t st[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(st, base + plan->o_stats, sizeof st, hipMemcpyDeviceToHost, ctx->stream));
  if (n && out) HIPCHK(hipMemcpyAsync(out, base + plan->o_out, sizeof(kp_launch_result) * n, hipMemcpyDeviceToHost, ctx->stream));
  if (n && out_types)
    HIPCHK(hipMemcpyAsync(out_types, base + plan->o_types, sizeof(uint32_t) * (size_t)n * plan->max_types,
                          hipMemcpyDeviceToHost, ctx->stream));
  if (n && out_overrides)
    HIPCHK(hipMemcpyAsync(out_overrides, base + plan->o_ovr, sizeof(uint32_t) * (size_t)n * plan->ovr_stride,
                          hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->device_ms = ms;
    stats->attempts = st[0];           // (request, listed type) pairs evaluated
    stats->bytes_algorithmic = st[1];
    stats->prepare_ms = plan->prepare_ms;
    stats->host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return KP_OK;
}

// ICE refresh of a prepared launch plan (same offering section as kp_filter_refresh; the offering -> class map and
// the subnet-zone classes do not change with availability or price).
int32_t kp_launch_refresh(kp_launch_plan* plan, const kp_catalog* cat) {
  if (!plan || !cat) return fail(KP_E_INVAL, "null argument");
  if (int32_t rc = CatalogsAlive({plan->alive})) return rc;
  if (cat != plan->cat || (int)cat->types.size() != plan->T)
    return fail(KP_E_INVAL, "kp_launch_refresh: the plan was prepared on another catalogue");
  int32_t rc = RefreshOfferings(plan->ctx, cat, plan->cp, plan->coff, (uint8_t*)plan->buf.p);
  if (rc != KP_OK) return rc;
  {  // the reservation tables follow availability and price too
    std::lock_guard<std::recursive_mutex> lock(plan->ctx->mu);
    map<ClassKey, int> cls_id;
    for (int c = 0; c < plan->cp.B->C; c++) cls_id[KeyOfClass(plan->cp.B->classes[c])] = c;
    vector<double> price_all;
    vector<int32_t> rcap;
    FillReservationTables(plan->cp.B->d, cat->types, cls_id, plan->cp.B->C, price_all, rcap);
    uint8_t* base = (uint8_t*)plan->buf.p;
    HIPCHK(hipMemcpyAsync(base + plan->o_pall, price_all.data(), price_all.size() * sizeof(double),
                          hipMemcpyHostToDevice, plan->ctx->stream));
    HIPCHK(hipMemcpyAsync(base + plan->o_rcap, rcap.data(), rcap.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                          plan->ctx->stream));
    HIPCHK(hipStreamSynchronize(plan->ctx->stream));
  }
  plan->seqnum = cat->seqnum;
  return KP_OK;
}

void kp_launch_plan_destroy(kp_launch_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  delete p;
}

int32_t kp_launch_select(kp_ctx* ctx, const kp_catalog* cat, const kp_launch_request* reqs, uint32_t n,
                         const char* const* subnet_zones, uint32_t n_subnet_zones, uint32_t max_types,
                         kp_launch_result* out, uint32_t* out_types, uint32_t* out_overrides, kp_solve_stats* stats) {
  if (!out) return fail(KP_E_INVAL, "null argument");
  kp_launch_plan* plan = nullptr;
  int32_t rc = kp_launch_prepare(ctx, cat, reqs, n, subnet_zones, n_subnet_zones, max_types, &plan);
  if (rc) return rc;
  rc = kp_launch_run(plan, out, out_types, out_overrides, stats);
  kp_launch_plan_destroy(plan);
  return rc;
}

// ---- consolidation: cluster snapshot + batched simulations -----------------------------------------
}  // extern "C"

// Owned deep copy of a kp_cluster (strings and nested arrays), kept by a cluster plan whose simulations run as
// whole Solves (the general path): the caller's buffers are not retained past kp_cluster_prepare.
struct OwnedCluster {
  std::deque<string> strs;
  vector<std::unique_ptr<uint8_t[]>> blocks;
  kp_cluster cl;
  vector<const kp_catalog*> cats;
  vector<std::shared_ptr<bool>> alive;
  const char* S(const char* x) {
    if (!x) return nullptr;
    strs.emplace_back(x);
    return strs.back().c_str();
  }
  template <class T>
  T* A(const T* src, size_t n) {
    if (!src || !n) return nullptr;
    blocks.emplace_back(new uint8_t[sizeof(T) * n]);
    T* d = reinterpret_cast<T*>(blocks.back().get());
    memcpy((void*)d, (const void*)src, sizeof(T) * n);
    return d;
  }
  void Reqs(kp_requirements& r) {
    kp_requirement* it = A(r.items, r.n);
    for (uint32_t i = 0; it && i < r.n; i++) {
      it[i].key = S(it[i].key);
      const char** v = (const char**)A(it[i].values, it[i].n_values);
      for (uint32_t j = 0; v && j < it[i].n_values; j++) v[j] = S(v[j]);
      it[i].values = v;
    }
    r.items = it;
  }
  const kp_label* Labels(const kp_label* l, uint32_t n) {
    kp_label* o = A(l, n);
    for (uint32_t i = 0; o && i < n; i++) o[i].key = S(o[i].key), o[i].value = S(o[i].value);
    return o;
  }
  const kp_taint* Taints(const kp_taint* t, uint32_t n) {
    kp_taint* o = A(t, n);
    for (uint32_t i = 0; o && i < n; i++) o[i].key = S(o[i].key), o[i].value = S(o[i].value);
    return o;
  }
  const kp_host_port* Ports(const kp_host_port* h, uint32_t n) {
    kp_host_port* o = A(h, n);
    for (uint32_t i = 0; o && i < n; i++) o[i].ip = S(o[i].ip);
    return o;
  }
  void Selector(kp_label_selector& s) {
    s.match_labels = Labels(s.match_labels, s.n_match_labels);
    kp_selector_requirement* e = A(s.match_expressions, s.n_match_expressions);
    for (uint32_t i = 0; e && i < s.n_match_expressions; i++) {
      e[i].key = S(e[i].key);
      const char** v = (const char**)A(e[i].values, e[i].n_values);
      for (uint32_t j = 0; v && j < e[i].n_values; j++) v[j] = S(v[j]);
      e[i].values = v;
    }
    s.match_expressions = e;
  }
  const kp_pod_affinity_term* Terms(const kp_pod_affinity_term* t, uint32_t n) {
    kp_pod_affinity_term* o = A(t, n);
    for (uint32_t i = 0; o && i < n; i++) {
      o[i].topology_key = S(o[i].topology_key);
      Selector(o[i].selector);
      Selector(o[i].namespace_selector);
      const char** v = (const char**)A(o[i].namespaces, o[i].n_namespaces);
      for (uint32_t j = 0; v && j < o[i].n_namespaces; j++) v[j] = S(v[j]);
      o[i].namespaces = v;
    }
    return o;
  }
  void Node(kp_existing_node& n) {
    n.name = S(n.name);
    n.labels = Labels(n.labels, n.n_labels);
    n.taints = Taints(n.taints, n.n_taints);
    n.host_ports = Ports(n.host_ports, n.n_host_ports);
  }
  explicit OwnedCluster(const kp_cluster* in) {
    cl = *in;
    cats.assign(in->catalogs, in->catalogs + in->n_catalogs);
    for (auto* c : cats) alive.push_back(c->alive);
    cl.catalogs = cats.data();
    cl.catalog_descs = nullptr;
    kp_nodepool* np = A(in->nodepools, in->n_nodepools);
    for (uint32_t i = 0; np && i < in->n_nodepools; i++) {
      np[i].name = S(np[i].name);
      Reqs(np[i].requirements);
      np[i].labels = Labels(np[i].labels, np[i].n_labels);
      np[i].taints = Taints(np[i].taints, np[i].n_taints);
    }
    cl.nodepools = np;
    kp_cluster_node* nd = A(in->nodes, in->n_nodes);
    for (uint32_t i = 0; nd && i < in->n_nodes; i++) {
      Node(nd[i].node);
      nd[i].pods = A(nd[i].pods, nd[i].n_pods);
    }
    cl.nodes = nd;
    kp_pod_shape* sh = A(in->shapes, in->n_shapes);
    for (uint32_t i = 0; sh && i < in->n_shapes; i++) {
      kp_pod_shape& x = sh[i];
      x.node_selector = Labels(x.node_selector, x.n_node_selector);
      kp_requirements* rt = A(x.required_terms, x.n_required_terms);
      for (uint32_t j = 0; rt && j < x.n_required_terms; j++) Reqs(rt[j]);
      x.required_terms = rt;
      kp_preferred_term* pt = A(x.preferred_terms, x.n_preferred_terms);
      for (uint32_t j = 0; pt && j < x.n_preferred_terms; j++) Reqs(pt[j].preference);
      x.preferred_terms = pt;
      kp_toleration* tl = A(x.tolerations, x.n_tolerations);
      for (uint32_t j = 0; tl && j < x.n_tolerations; j++) tl[j].key = S(tl[j].key), tl[j].value = S(tl[j].value);
      x.tolerations = tl;
      kp_topology_spread* ts = A(x.topology_spread, x.n_topology_spread);
      for (uint32_t j = 0; ts && j < x.n_topology_spread; j++) {
        ts[j].topology_key = S(ts[j].topology_key);
        Selector(ts[j].selector);
      }
      x.topology_spread = ts;
      x.namespace_ = S(x.namespace_);
      x.labels = Labels(x.labels, x.n_labels);
      x.host_ports = Ports(x.host_ports, x.n_host_ports);
      kp_requirements vr{x.volume_requirements, x.n_volume_requirements, 0};
      Reqs(vr);
      x.volume_requirements = vr.items;
      x.required_anti_affinity = Terms(x.required_anti_affinity, x.n_required_anti_affinity);
      x.preferred_anti_affinity = Terms(x.preferred_anti_affinity, x.n_preferred_anti_affinity);
      x.required_affinity = Terms(x.required_affinity, x.n_required_affinity);
      x.preferred_affinity = Terms(x.preferred_affinity, x.n_preferred_affinity);
    }
    cl.shapes = sh;
    kp_pod* pods = A(in->pods, in->n_pods);
    if (in->pod_uids && pods) {  // each subset's Solve sees the pods' exact UID ranks as their keys
      vector<uint64_t> k;
      if (ExactUidKeys(in->pod_uids, in->n_pods, k))
        for (uint32_t i = 0; i < in->n_pods; i++) pods[i].uid_key = k[i];
    }
    cl.pods = pods;
    cl.pod_uids = nullptr;
    cl.pending_pods = A(in->pending_pods, in->n_pending);
    kp_namespace* ns = A(in->namespaces, in->n_namespaces);
    for (uint32_t i = 0; ns && i < in->n_namespaces; i++) ns[i].name = S(ns[i].name), ns[i].labels = Labels(ns[i].labels, ns[i].n_labels);
    cl.namespaces = ns;
  }
};

struct GeneralBatch;
struct kp_cluster_plan {
  CtxRef ctx;
  std::unique_ptr<OwnedCluster> general;  // set: simulations run as whole Solves (kp_solve on this device)
  double general_ms = 0;                  // device time of the last general batch (solve + finalize kernels)
  uint64_t general_phase[8] = {};         // kp_overrides.timing: the batch's solve_kernel phase cycles, summed
  std::shared_ptr<GeneralBatch> gb;       // the general path's superset Solve (batched simulations), once built
  vector<std::map<string, string>> general_labels;
  bool gb_tried = false;
  uint32_t general_batched = 0;           // simulations of the last general batch that ran batched
  std::unique_ptr<Compiled> cp;
  DevBuf buf;                       // resident snapshot
  DevBuf scratch;                   // per-wave state, grown on demand
  size_t scratch_bytes = 0;
  DevBuf batch;                     // subsets + results, grown on demand
  size_t batch_bytes = 0;
  SimArgs a;
  int N = 0, T2 = 1, n_cu = 256;
  vector<uint32_t> node_npods;
  vector<uint8_t> deleting;         // [N] MarkedForDeletion
  int n_base = 0;                   // pending + deleting-node pods in every simulation
  double prepare_ms = 0;
  // kp_cluster_refresh: where the offering-dependent parts live in the snapshot, and what they derive from
  vector<CatOffsets> coffs;
  size_t o_tX = 0, o_nprice = 0, o_nflags = 0;
  struct NodeOffer {
    uint32_t cat, type;
    std::map<string, string> labels;  // the capacity-type / zone / zone-id labels (NodeCandidatePrice)
  };
  vector<NodeOffer> node_offer;
  vector<uint8_t> node_flags;
};

namespace {
static_assert(sizeof(SimOut) == sizeof(kp_sim_result), "SimOut mirrors kp_sim_result");

// Offerings.Compatible(NewLabelRequirements(node labels)).Cheapest().Price: an offering's capacity-type /
// zone / zone-id requirement (all well-known) is compatible unless the node carries that label with a
// different value.
bool NodeCandidatePrice(const HostType& t, const std::map<string, string>& labels, double* price) {
  bool any = false;
  double p = 0;
  auto clash = [&](const char* key, bool has, const string& v) {
    if (!has) return false;
    auto f = labels.find(key);
    return f != labels.end() && f->second != v;
  };
  // the reservation keys: an offering without one requires DoesNotExist (R:offering.go:136-137), so a node labelled
  // with a reservation id / type is compatible only with the offerings of that reservation
  auto clash_res = [&](const char* key, bool has, const string& v) {
    auto f = labels.find(key);
    if (f == labels.end()) return false;
    return !has || f->second != v;
  };
  for (auto& o : t.offs) {
    if (clash(kCapType, true, o.ct) || clash(kZone, o.has_zone, o.zone) || clash(kZoneID, o.has_zid, o.zid)) continue;
    if (clash_res(kResID, o.has_rid, o.rid) || clash_res(kResType, o.has_rt, o.rt)) continue;
    if (!any || o.price < p) p = o.price;
    any = true;
  }
  *price = p;
  return any;
}
}  // namespace

extern "C" {

struct GeneralBatch;
static int32_t GeneralBatchBuild(kp_cluster_plan* plan, std::shared_ptr<GeneralBatch>& out);
// A cluster plan for the general path: the cluster is kept as an owned copy and compiled as the batched simulations'
// superset Solve (or, where that does not apply, validated by a host compile: every node existing, every pod pending).
static int32_t PrepareGeneral(kp_ctx* ctx, const kp_cluster* cl, kp_cluster_plan** out,
                              std::chrono::steady_clock::time_point t0) {
  for (uint32_t i = 0; i < cl->n_catalogs; i++)
    if (!cl->catalogs || !cl->catalogs[i]) return fail(KP_E_INVAL, "catalogue %u is null", i);
  vector<kp_existing_node> ex(cl->n_nodes);
  for (uint32_t i = 0; i < cl->n_nodes; i++) ex[i] = cl->nodes[i].node;
  kp_solve_in in;
  memset(&in, 0, sizeof in);
  in.catalogs = cl->catalogs;
  in.n_catalogs = cl->n_catalogs;
  in.n_nodepools = cl->n_nodepools;
  in.nodepools = cl->nodepools;
  in.existing = ex.data();
  in.n_existing = cl->n_nodes;
  in.n_shapes = cl->n_shapes;
  in.shapes = cl->shapes;
  in.pods = cl->pods;
  in.n_pods = cl->n_pods;
  in.max_instance_types = 100;
  in.namespaces = cl->namespaces;
  in.n_namespaces = cl->n_namespaces;
  in.pod_uids = cl->pod_uids;
  PhaseTimer pt;
  auto plan = std::make_unique<kp_cluster_plan>();
  plan->ctx = ctx;
  plan->N = (int)cl->n_nodes;
  plan->general = std::make_unique<OwnedCluster>(cl);
  pt.lap("general: owned copy");
  // the superset Solve of the batched simulations, built now (it validates every node and pod as well); a cluster
  // it does not take keeps the per-subset compile, validated here by the whole-cluster compile
  int32_t rc = KP_E_UNSUPPORTED;
  if (ctx->ov.general_batch == 0) {
    std::lock_guard<std::recursive_mutex> lock(ctx->mu);
    HIPCHK(hipSetDevice(ctx->device));
    plan->gb_tried = true;
    rc = GeneralBatchBuild(plan.get(), plan->gb);
    // the batched layout is an optimisation: a device that cannot hold it leaves the per-subset compile
    if (rc == KP_E_NOMEM || rc == KP_E_DEVICE) (void)hipGetLastError(), rc = KP_E_UNSUPPORTED;
    if (rc && rc != KP_E_UNSUPPORTED) return rc;
    if (rc) plan->gb.reset();
  }
  if (rc) {
    Compiled C;
    rc = CompileSolve(&in, C);
    if (rc) return rc;
  }
  plan->prepare_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = plan.release();
  return KP_OK;
}

int32_t kp_cluster_prepare(kp_ctx* ctx, const kp_cluster* cl, kp_cluster_plan** out) {
  auto t0 = std::chrono::steady_clock::now();
  if (!ctx || !cl || !out) return fail(KP_E_INVAL, "null argument");
  if (cl->n_nodes && !cl->nodes) return fail(KP_E_INVAL, "null nodes");
  if (cl->pod_uids)  // one rule on every path (batched kernels, general batch, per-subset compile): as kp_solve
    for (uint32_t i = 0; i < cl->n_pods; i++)
      if (!cl->pod_uids[i]) return fail(KP_E_INVAL, "null pod uid");
  // capacity reservations: SimulateScheduling's Solve reserves offerings strictly (DisableReservedCapacityFallback),
  // which the batched kernels do not model: such clusters take the general path (whole device Solves)
  bool topo = false;
  for (uint32_t i = 0; i < cl->n_catalogs; i++)
    topo |= cl->catalogs && cl->catalogs[i] && cl->catalogs[i]->reservations;
  for (uint32_t i = 0; i < cl->n_shapes; i++)
    topo |= cl->shapes[i].n_topology_spread > 0 || PodTermCount(cl->shapes[i]) > 0;
  {  // a pod requirement on kubernetes.io/hostname (the batched kernels' node compatibility drops the hostname)
    std::set<string> named;
    for (uint32_t i = 0; i < cl->n_shapes && !topo; i++) {
      const kp_pod_shape& sh = cl->shapes[i];
      for (uint32_t j = 0; j < sh.n_node_selector; j++)
        topo |= sh.node_selector[j].key && string(sh.node_selector[j].key) == kHostname;
      for (uint32_t j = 0; j < sh.n_required_terms; j++) HostnameNames(sh.required_terms[j], &topo, &named);
      for (uint32_t j = 0; j < sh.n_preferred_terms; j++) HostnameNames(sh.preferred_terms[j].preference, &topo, &named);
      HostnameNames(kp_requirements{sh.volume_requirements, sh.n_volume_requirements, 0}, &topo, &named);
    }
  }
  if (topo) return PrepareGeneral(ctx, cl, out, t0);
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  auto plan = std::make_unique<kp_cluster_plan>();
  plan->ctx = ctx;
  plan->cp = std::make_unique<Compiled>();
  Compiled& C = *plan->cp;
  const int N = (int)cl->n_nodes;
  plan->N = N;
  vector<kp_existing_node> ex(N);
  for (int i = 0; i < N; i++) ex[i] = cl->nodes[i].node;
  kp_solve_in in;
  memset(&in, 0, sizeof in);
  in.catalogs = cl->catalogs;
  in.n_catalogs = cl->n_catalogs;
  in.n_nodepools = cl->n_nodepools;
  in.nodepools = cl->nodepools;
  in.existing = ex.data();
  in.n_existing = (uint32_t)N;
  in.n_shapes = cl->n_shapes;
  in.shapes = cl->shapes;
  in.pods = cl->pods;
  in.n_pods = cl->n_pods;
  in.max_instance_types = 100;
  in.namespaces = cl->namespaces;
  in.n_namespaces = cl->n_namespaces;
  in.pod_uids = cl->pod_uids;
  int32_t rc = CompileSolve(&in, C);
  if (rc) return rc;
  const Dict& d = C.B->d;
  const int TW = C.B->TW, E = N, EW = (E + 63) / 64, SL = (int)C.shape_reqs.size(), NT = (int)C.B->tmpl_reqs.size();
  const int T = d.dd.T, K = d.dd.K;
  // a pod NotIn/DoesNotExist on a key some node lacks would add that key to the node's requirements
  uint64_t all_nodes_keys = ~0ull;
  for (auto& q : C.ex_reqs) all_nodes_keys &= q.present;
  for (int sl = 0; sl < SL; sl++)
    if (C.shape_negop[sl] & ~all_nodes_keys)  // CanAdd is then not a function of the snapshot: whole Solves
      return PrepareGeneral(ctx, cl, out, t0);
  // existing nodes: label value bit per key (node labels are single-valued In requirements)
  vector<uint16_t> ex_code((size_t)std::max(K, 1) * std::max(E, 1), 0xFFFF);
  vector<uint8_t> ex_init(std::max(E, 1), 0);
  vector<int32_t> node_pos(std::max(N, 1), 0);
  for (int e = 0; e < E; e++) {
    const KReqs& q = C.ex_reqs[e];
    node_pos[C.ex_input[e]] = e;
    ex_init[e] = cl->nodes[C.ex_input[e]].node.initialized ? 1 : 0;
    for (int k = 0; k < K; k++) {
      if (!((q.present >> k) & 1)) continue;
      for (int wi = 0; wi < nwords(d, k); wi++) {
        const int w = kw(d, k, wi);
        if (q.vals[w]) {
          ex_code[(size_t)k * E + e] = (uint16_t)(w * 64 + __builtin_ctzll(q.vals[w]));
          break;
        }
      }
    }
  }
  // pods: global queue rank
  const uint32_t P = cl->n_pods;
  vector<uint32_t> rank(std::max<uint32_t>(P, 1)), rank_pod(std::max<uint32_t>(P, 1));
  for (uint32_t i = 0; i < P; i++) {
    rank[C.queue[i]] = i;
    rank_pod[i] = (uint32_t)C.queue[i];
  }
  // cluster nodes: pods (CSR), candidate price, flags, type-name ids
  std::unordered_map<string, uint32_t> names;
  auto name_id = [&](const string& s) {
    auto it = names.find(s);
    if (it != names.end()) return it->second;
    const uint32_t id = (uint32_t)names.size();
    names[s] = id;
    return id;
  };
  vector<uint32_t> node_off(N + 1, 0), node_pods;
  vector<double> node_price(std::max(N, 1), 0);
  vector<uint8_t> node_flags(std::max(N, 1), 0);
  vector<uint32_t> node_name(std::max(N, 1), 0);
  plan->node_npods.resize(N);
  for (int i = 0; i < N; i++) {
    const kp_cluster_node& n = cl->nodes[i];
    if (n.catalog >= cl->n_catalogs || !cl->catalogs[n.catalog]) return fail(KP_E_INVAL, "node %d: catalogue %u", i, n.catalog);
    const kp_catalog* cat = cl->catalogs[n.catalog];
    if (n.instance_type >= cat->types.size()) return fail(KP_E_INVAL, "node %d: instance type %u", i, n.instance_type);
    if (n.n_pods && !n.pods) return fail(KP_E_INVAL, "node %d: null pods", i);
    for (uint32_t j = 0; j < n.n_pods; j++) {
      if (n.pods[j] >= P) return fail(KP_E_INVAL, "node %d: pod %u", i, n.pods[j]);
      node_pods.push_back(n.pods[j]);
    }
    node_off[i + 1] = (uint32_t)node_pods.size();
    plan->node_npods[i] = n.n_pods;
    std::map<string, string> labels;
    for (uint32_t j = 0; j < n.node.n_labels; j++)
      labels[Normalize(n.node.labels[j].key ? n.node.labels[j].key : "")] = n.node.labels[j].value ? n.node.labels[j].value : "";
    const HostType& ht = cat->types[n.instance_type];
    double pr = 0;
    const bool priced = NodeCandidatePrice(ht, labels, &pr);
    node_price[i] = pr;
    auto ct = labels.find(kCapType);
    node_flags[i] = (priced ? 1 : 0) | (ct != labels.end() && ct->second == "spot" ? 2 : 0);
    node_name[i] = name_id(ht.name);
    kp_cluster_plan::NodeOffer no{n.catalog, n.instance_type, {}};
    for (const char* k : {kCapType, kZone, kZoneID}) {
      auto f = labels.find(k);
      if (f != labels.end()) no.labels[k] = f->second;
    }
    plan->node_offer.push_back(std::move(no));
  }
  if (node_pods.empty()) node_pods.push_back(0);
  // pods every simulation schedules besides those of S (SimulateScheduling: pending pods and the pods of nodes
  // already being deleted), and the deleting nodes, which are never destinations
  if (cl->n_pending && !cl->pending_pods) return fail(KP_E_INVAL, "null pending_pods");
  vector<uint8_t> pod_kind(std::max<uint32_t>(P, 1), 0);
  vector<uint32_t> base_keys;
  vector<uint64_t> base_excl(std::max(EW, 1), 0);
  plan->deleting.assign(N, 0);
  for (uint32_t j = 0; j < cl->n_pending; j++) {
    const uint32_t p = cl->pending_pods[j];
    if (p >= P) return fail(KP_E_INVAL, "pending pod %u", p);
    if (pod_kind[p]) return fail(KP_E_INVAL, "pod %u listed twice", p);
    pod_kind[p] = 2;
    base_keys.push_back(rank[p]);
  }
  for (int i = 0; i < N; i++) {
    if (!cl->nodes[i].deleting) continue;
    plan->deleting[i] = 1;
    const int e = node_pos[i];
    base_excl[e >> 6] |= 1ull << (e & 63);
    for (uint32_t j = node_off[i]; j < node_off[i + 1]; j++) {
      if (pod_kind[node_pods[j]]) return fail(KP_E_INVAL, "pod %u listed twice", node_pods[j]);
      pod_kind[node_pods[j]] = 1;
      base_keys.push_back(rank[node_pods[j]]);
    }
  }
  plan->n_base = (int)base_keys.size();
  if (base_keys.empty()) base_keys.push_back(0);
  vector<uint32_t> type_name((size_t)cl->n_catalogs * std::max(T, 1), 0xFFFFFFFFu);
  for (uint32_t c = 0; c < cl->n_catalogs; c++)
    for (size_t t = 0; t < cl->catalogs[c]->types.size(); t++)
      type_name[(size_t)c * T + t] = name_id(cl->catalogs[c]->types[t].name);
  vector<int32_t> sl_shape(std::max(SL, 1), 0);
  for (uint32_t s = 0; s < cl->n_shapes; s++)
    for (int l = 0; l < C.shape_nlevels[s]; l++) sl_shape[C.shape_level_base[s] + l] = (int32_t)s;
  const int ctk = d.key(kCapType);

  Blob blob;
  const size_t o_dict = blob.put(&C.B->d.dd, 1);
  const size_t o_vint = blob.put(C.B->d.vint);
  vector<CatOffsets> coffs;
  PutCatalogs(blob, C, coffs);
  const size_t o_cats = blob.reserve(sizeof(DevCatalog) * coffs.size());
  const size_t o_slb = blob.put(C.shape_level_base);
  const size_t o_snl = blob.put(C.shape_nlevels);
  const size_t o_sls = blob.put(sl_shape);
  const size_t o_sreqs = blob.put(C.shape_reqs);
  const size_t o_sneg = blob.put(C.shape_negop);
  const size_t o_sreq = blob.put(C.shape_requests);
  const size_t o_stol = blob.put(C.shape_tolerates);
  const size_t o_pvp = blob.put(C.pvp);
  const size_t o_pvpb = blob.put(C.pvp_base);
  const size_t o_pvps = blob.put(C.pvp_slot);
  vector<int32_t> tmpl_np(C.B->tmpl_nodepool.begin(), C.B->tmpl_nodepool.end());
  if (tmpl_np.empty()) tmpl_np.push_back(0);
  const size_t o_treqs = blob.put(C.B->tmpl_reqs);
  const size_t o_tts = blob.put(C.B->tmpl_taintset);
  const size_t o_tcat = blob.put(C.B->tmpl_catalog);
  const size_t o_tnp = blob.put(tmpl_np);
  const size_t o_tX = blob.put(C.B->tmpl_X);
  const size_t o_tdm = blob.put(C.B->tmpl_daemon);
  const size_t o_excode = blob.put(ex_code);
  const size_t o_exts = blob.put(C.ex_taintset);
  const size_t o_exav = blob.put(C.ex_available);
  const size_t o_exrq = blob.put(C.ex_requests);
  const size_t o_exin = blob.put(ex_init);
  const size_t o_pshape = blob.put(C.pod_shape);
  const size_t o_prank = blob.put(rank);
  const size_t o_rpod = blob.put(rank_pod);
  const size_t o_npos = blob.put(node_pos);
  const size_t o_noff = blob.put(node_off);
  const size_t o_npods = blob.put(node_pods);
  const size_t o_nprice = blob.put(node_price);
  const size_t o_nflags = blob.put(node_flags);
  const size_t o_nname = blob.put(node_name);
  const size_t o_tname = blob.put(type_name);
  const size_t o_pkind = blob.put(pod_kind);
  const size_t o_bkeys = blob.put(base_keys);
  const size_t o_bexcl = blob.put(base_excl);
  const size_t o_tlp = blob.put(C.tmpl_limit_present);
  const size_t o_trem = blob.put(C.tmpl_remaining);
  const size_t o_shpc = blob.put(C.shape_hp_conf), o_shpa = blob.put(C.shape_hp_add), o_exhp = blob.put(C.ex_hp);
  const size_t host_bytes = blob.host.size();
  const size_t o_usable = blob.reserve(sizeof(uint64_t) * (size_t)std::max(SL, 1) * std::max(EW, 1));
  const size_t o_tres = blob.reserve(sizeof(SimNC) * (size_t)std::max(SL, 1));
  HIPCHK(hipMalloc(&plan->buf.p, blob.host.size()));
  uint8_t* base = (uint8_t*)plan->buf.p;
  {
    vector<DevCatalog> dc = DevCats(base, C, coffs);
    memcpy(blob.host.data() + o_cats, dc.data(), sizeof(DevCatalog) * dc.size());
  }
  HIPCHK(hipMemcpyAsync(base, blob.host.data(), host_bytes, hipMemcpyHostToDevice, ctx->stream));

  SimArgs& a = plan->a;
  memset(&a, 0, sizeof a);
  a.dict = (const DevDict*)(base + o_dict);
  a.cats = (const DevCatalog*)(base + o_cats);
  a.n_catalogs = (int32_t)coffs.size();
  a.SL = SL;
  a.vint = (const int64_t*)(base + o_vint);
  a.shape_level_base = (const int32_t*)(base + o_slb);
  a.shape_nlevels = (const int32_t*)(base + o_snl);
  a.sl_shape = (const int32_t*)(base + o_sls);
  a.shape_reqs = base + o_sreqs;
  a.shape_negop = (const uint64_t*)(base + o_sneg);
  a.shape_requests = (const int64_t*)(base + o_sreq);
  a.shape_tolerates = (const uint64_t*)(base + o_stol);
  a.shape_pvp = (const uint64_t*)(base + o_pvp);
  a.pvp_base = (const int32_t*)(base + o_pvpb);
  a.pvp_slot = (const int32_t*)(base + o_pvps);
  a.n_tmpl = NT;
  a.tmpl_reqs = base + o_treqs;
  a.tmpl_taintset = (const int32_t*)(base + o_tts);
  a.tmpl_catalog = (const int32_t*)(base + o_tcat);
  a.tmpl_nodepool = (const int32_t*)(base + o_tnp);
  a.tmpl_X = (const uint64_t*)(base + o_tX);
  a.tmpl_daemon = (const int64_t*)(base + o_tdm);
  a.tmpl_limit_present = (const uint32_t*)(base + o_tlp);
  a.tmpl_remaining = (const int64_t*)(base + o_trem);
  a.pod_kind = base + o_pkind;
  a.base_keys = (const uint32_t*)(base + o_bkeys);
  a.base_excl = (const uint64_t*)(base + o_bexcl);
  a.n_base = plan->n_base;
  a.E = E;
  a.EW = EW;
  a.ex_code = (const uint16_t*)(base + o_excode);
  a.ex_taintset = (const int32_t*)(base + o_exts);
  a.ex_available = (const int64_t*)(base + o_exav);
  a.ex_requests = (const int64_t*)(base + o_exrq);
  a.ex_init = base + o_exin;
  a.hp_any = C.hp_any ? 1 : 0;
  a.shape_hp_conf = (const uint64_t*)(base + o_shpc);
  a.shape_hp_add = (const uint64_t*)(base + o_shpa);
  a.ex_hp = (const uint64_t*)(base + o_exhp);
  a.usable = (uint64_t*)(base + o_usable);
  a.tres = (SimNC*)(base + o_tres);
  a.pod_shape = (const int32_t*)(base + o_pshape);
  a.pod_rank = (const uint32_t*)(base + o_prank);
  a.rank_pod = (const uint32_t*)(base + o_rpod);
  a.node_pos = (const int32_t*)(base + o_npos);
  a.node_pod_off = (const uint32_t*)(base + o_noff);
  a.node_pods = (const uint32_t*)(base + o_npods);
  a.node_price = (const double*)(base + o_nprice);
  a.node_flags = base + o_nflags;
  a.node_name = (const uint32_t*)(base + o_nname);
  a.type_name = (const uint32_t*)(base + o_tname);
  a.ct_key = ctk;
  a.spot_bit = ctk >= 0 ? d.bit(ctk, "spot") : -1;
  a.od_bit = ctk >= 0 ? d.bit(ctk, "on-demand") : -1;
  a.req_res_mask = 0;
  for (size_t i = 0; i < C.shape_requests.size(); i++)
    if (C.shape_requests[i] > 0) a.req_res_mask |= 1u << (i % KP_NRES);
  for (size_t i = 0; i < C.B->tmpl_daemon.size(); i++)
    if (C.B->tmpl_daemon[i] > 0) a.req_res_mask |= 1u << (i % KP_NRES);
  a.RU = 0;
  for (int r = 0; r < KP_NRES; r++)
    if ((a.req_res_mask >> r) & 1) a.ru_res[a.RU++] = (int8_t)r;
  a.max_types = 100;
  a.spot_to_spot = cl->spot_to_spot ? 1 : 0;
  (void)TW;
  plan->T2 = 1;
  while (plan->T2 < std::max(T, 1)) plan->T2 <<= 1;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess && ncu > 0)
    plan->n_cu = ncu;
  plan->coffs = coffs;
  plan->o_tX = o_tX;
  plan->o_nprice = o_nprice;
  plan->o_nflags = o_nflags;
  plan->node_flags = node_flags;
  HIPCHK(launch_sim_prep(a, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  plan->prepare_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = plan.release();
  return KP_OK;
}

// ICE refresh of a resident snapshot (kp_cluster_refresh, see kp_solve_refresh): the catalogues' offering arrays,
// the templates' options, the candidates' prices, then sim_prep_kernel again (its per shape-level template
// outcomes read the options and prices). A general-path plan compiles every simulation from the live catalogues.
int32_t kp_cluster_refresh(kp_cluster_plan* plan) {
  if (!plan) return fail(KP_E_INVAL, "null argument");
  if (plan->general) return KP_OK;
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  SolveBase& B = *plan->cp->B;
  if (int32_t rc = CatalogsAlive(B.alive)) return rc;
  if (SeqnumsOf(B.catalogs) == B.seqnums) return KP_OK;
  // host side; the snapshot's own device copy is written below, and the new seqnums are committed only once it is
  int32_t rc = RefreshOfferings(nullptr, B, false);
  if (rc < 0) return rc;
  if (rc > 0) return fail(KP_E_INVAL, "the offering update changed which NodePools keep instance types: prepare again");
  uint8_t* base = (uint8_t*)plan->buf.p;
  hipStream_t st = ctx->stream;
  for (size_t i = 0; i < B.cats.size(); i++) {
    const HostCat& hc = B.cats[i];
    const CatOffsets& o = plan->coffs[i];
    HIPCHK(hipMemcpyAsync(base + o.offer, hc.offer_avail.data(), hc.offer_avail.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(base + o.price, hc.price.data(), hc.price.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(base + o.price_cm, hc.price_cm.data(), hc.price_cm.size() * 8, hipMemcpyHostToDevice, st));
    if (!hc.price_sub.empty())
      HIPCHK(hipMemcpyAsync(base + o.price_sub, hc.price_sub.data(), hc.price_sub.size() * 8, hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipMemcpyAsync(base + plan->o_tX, B.tmpl_X.data(), B.tmpl_X.size() * 8, hipMemcpyHostToDevice, st));
  vector<double> price(std::max<size_t>(plan->node_offer.size(), 1), 0);
  for (size_t i = 0; i < plan->node_offer.size(); i++) {
    const auto& no = plan->node_offer[i];
    const bool priced = NodeCandidatePrice(B.catalogs[no.cat]->types[no.type], no.labels, &price[i]);
    plan->node_flags[i] = (uint8_t)((plan->node_flags[i] & ~1) | (priced ? 1 : 0));
  }
  HIPCHK(hipMemcpyAsync(base + plan->o_nprice, price.data(), price.size() * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(base + plan->o_nflags, plan->node_flags.data(), plan->node_flags.size(), hipMemcpyHostToDevice, st));
  HIPCHK(launch_sim_prep(plan->a, st));
  HIPCHK(hipStreamSynchronize(st));
  CommitRefresh(B);
  return KP_OK;
}

void kp_cluster_plan_destroy(kp_cluster_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  delete p;
}

// One batch on the resident snapshot, results left on the device (a_out.out); the caller holds ctx->mu.
// ---- general simulations: each subset's SimulateScheduling as a whole Solve on the device -----------------------
// Used for clusters the batched sim kernels do not model (topology spread; pod NotIn/DoesNotExist on a label key
// some node lacks). Per subset: the pending pods, the deleting nodes' pods and the subset's pods are scheduled onto
// every other node (existing), with every pod still bound to one of those nodes as a bound pod (Topology.countDomains
// skips the pods being scheduled), then computeConsolidation's decision is taken on the Solve result exactly as the
// batched kernel takes it (sim_kernel's decision; disruption.md:89-128).
namespace {
bool OfferAdmits(const Dict& d, const KReqs& R, const HostOffering& o) {
  auto admits = [&](const char* key, bool has, const string& v) {
    if (!has) return true;
    const int k = d.key(key);
    if (k < 0 || !((R.present >> k) & 1)) return true;  // undefined well-known key: allowed
    const int b = d.bit(k, v);
    if (b < 0) return ((R.compl_ >> k) & 1) != 0;
    return Has(d, R, k, b);
  };
  // reservation keys: an offering without one is DoesNotExist on it, compatible with NotIn / DoesNotExist only
  auto admits_res = [&](const char* key, bool has, const string& v) {
    if (has) return admits(key, true, v);
    const int k = d.key(key);
    if (k < 0 || !((R.present >> k) & 1)) return true;
    const bool c = ((R.compl_ >> k) & 1) != 0, nz = KeyNonEmptyVals(d, R, k);
    return (c && nz) || (!c && !nz);
  };
  return admits(kCapType, true, o.ct) && admits(kZone, o.has_zone, o.zone) && admits(kZoneID, o.has_zid, o.zid) &&
         admits_res(kResID, o.has_rid, o.rid) && admits_res(kResType, o.has_rt, o.rt);
}
// Offerings.Available().Compatible(reqs).WorstLaunchPrice: capacity types in precedence reserved, spot, on-demand
double WorstLaunch(const Dict& d, const KReqs& R, const HostType& t, bool spot_only) {
  for (const char* ct : {"reserved", "spot", "on-demand"}) {
    if (spot_only && strcmp(ct, "spot") != 0) continue;
    bool any = false;
    double mx = 0;
    for (auto& o : t.offs) {
      if (!o.available || o.ct != ct || !OfferAdmits(d, R, o)) continue;
      if (!any || o.price > mx) mx = o.price;
      any = true;
    }
    if (any) return mx;
  }
  return std::numeric_limits<double>::max();
}
}  // namespace

static int32_t SolvePrepare(kp_ctx* ctx, const kp_solve_in* in, kp_comm* comm, kp_solve_plan** out);

// The offerings as OfferAdmits reads them, resolved against one dictionary once (the batched decisions run
// WorstLaunch over up to 100 options per simulation): per offering its capacity-type class and the dictionary bits
// of its five offering keys (-1: a value the dictionary lacks, -2: the offering has no such requirement).
struct OffBits {
  int16_t ct_class;  // 0 reserved, 1 spot, 2 on-demand, 3 other
  int16_t b[5];      // capacity type, zone, zone id, reservation id, reservation type
};
struct OfferTab {
  int k[5];                                  // the five keys' dictionary ids (-1: absent)
  vector<vector<vector<OffBits>>> off;       // [catalogue][type][offering]
  void Build(const Dict& d, const kp_cluster& cl) {
    const char* keys[5] = {kCapType, kZone, kZoneID, kResID, kResType};
    for (int i = 0; i < 5; i++) k[i] = d.key(keys[i]);
    off.assign(cl.n_catalogs, {});
    for (uint32_t c = 0; c < cl.n_catalogs; c++) {
      const vector<HostType>& types = cl.catalogs[c]->types;
      off[c].resize(types.size());
      for (size_t t = 0; t < types.size(); t++)
        for (const HostOffering& o : types[t].offs) {
          OffBits x;
          x.ct_class = o.ct == "reserved" ? 0 : o.ct == "spot" ? 1 : o.ct == "on-demand" ? 2 : 3;
          const string* v[5] = {&o.ct, &o.zone, &o.zid, &o.rid, &o.rt};
          const bool has[5] = {true, o.has_zone, o.has_zid, o.has_rid, o.has_rt};
          for (int i = 0; i < 5; i++) x.b[i] = !has[i] ? -2 : k[i] < 0 ? -1 : (int16_t)std::max(-1, d.bit(k[i], *v[i]));
          off[c][t].push_back(x);
        }
    }
  }
  // OfferAdmits on the resolved bits
  bool Admits(const Dict& d, const KReqs& R, const OffBits& x) const {
    for (int i = 0; i < 5; i++) {
      const int kk = k[i];
      if (kk < 0 || !((R.present >> kk) & 1)) continue;  // undefined well-known key: allowed
      if (x.b[i] == -2) {
        if (i < 3) continue;  // no zone / zone-id requirement on the offering
        const bool c = ((R.compl_ >> kk) & 1) != 0, nz = KeyNonEmptyVals(d, R, kk);  // DoesNotExist on it
        if (!((c && nz) || (!c && !nz))) return false;
      } else if (x.b[i] == -1) {
        if (!((R.compl_ >> kk) & 1)) return false;
      } else if (!Has(d, R, kk, x.b[i])) {
        return false;
      }
    }
    return true;
  }
  // WorstLaunch on the resolved bits
  double Worst(const Dict& d, const KReqs& R, const HostType& t, const vector<OffBits>& ob, bool spot_only) const {
    for (int cls = 0; cls < 3; cls++) {
      if (spot_only && cls != 1) continue;
      bool any = false;
      double mx = 0;
      for (size_t i = 0; i < t.offs.size(); i++) {
        const HostOffering& o = t.offs[i];
        if (!o.available || ob[i].ct_class != cls || !Admits(d, R, ob[i])) continue;
        if (!any || o.price > mx) mx = o.price;
        any = true;
      }
      if (any) return mx;
    }
    return std::numeric_limits<double>::max();
  }
};

// getCandidatePrices' per-node terms, once per cluster plan (the nodes' labels and offerings do not change between
// batches; a catalogue refresh rebuilds the batch and with it this cache)
struct CandCache {
  vector<double> price;        // cheapest label-compatible offering price
  vector<char> priced, spot;   // some offering is compatible; the node is labelled spot
  void Build(const kp_cluster& cl, const vector<std::map<string, string>>& labels) {
    const int N = (int)cl.n_nodes;
    price.assign(N, 0);
    priced.assign(N, 0);
    spot.assign(N, 0);
    for (int c = 0; c < N; c++) {
      const kp_cluster_node& n = cl.nodes[c];
      double p = 0;
      priced[c] = NodeCandidatePrice(cl.catalogs[n.catalog]->types[n.instance_type], labels[c], &p) ? 1 : 0;
      price[c] = p;
      auto f = labels[c].find(kCapType);
      spot[c] = f != labels[c].end() && f->second == "spot";
    }
  }
};

// computeConsolidation's decision on one simulation's Solve (sim_kernel's decision; disruption.md:89-128). all: every
// non-pending pod was scheduled (and no candidate pod onto an uninitialized node). The Solve made n_nc NodeClaims;
// R / ci / nodepool / opts: the first one's final requirements (held reservation ids applied), catalogue, NodePool and
// price-ordered options (after Truncate), minValues not yet checked on them.
static void GeneralDecide(const kp_cluster& cl, const vector<std::map<string, string>>& labels,
                          const vector<uint32_t>& cand, const SolveBase& B, bool all, int n_nc, const KReqs* R,
                          int ci, uint32_t nodepool, const uint32_t* opts, uint32_t n_opts, int32_t multi_node,
                          SimOut& r, const OfferTab* tab = nullptr, const CandCache* cc = nullptr) {
  double candPrice = 0;
  bool priced = true, allSpot = true;
  for (uint32_t c : cand) {
    if (cc) {
      priced = priced && cc->priced[c];
      candPrice += cc->price[c];
      allSpot = allSpot && cc->spot[c];
      continue;
    }
    const kp_cluster_node& n = cl.nodes[c];
    double p = 0;
    if (!NodeCandidatePrice(cl.catalogs[n.catalog]->types[n.instance_type], labels[c], &p)) priced = false;
    candPrice += p;
    auto f = labels[c].find(kCapType);
    if (f == labels[c].end() || f->second != "spot") allSpot = false;
  }
  r.candidate_price = priced ? candPrice : 0;
  if (!all) return;  // no-op
  if (n_nc == 0) {
    r.decision = KP_DECISION_DELETE;
    r.savings = r.candidate_price;
    return;
  }
  if (n_nc != 1 || !priced) return;
  const Dict& d = B.d;
  const vector<HostType>& types = cl.catalogs[ci]->types;
  const HostCat& hc = B.cats[ci];
  const bool hasMin = (R->hmin & R->present) != 0;
  if (hasMin) {  // Truncate(reqs, max): minValues must hold on the truncated options, else its pods fail (no-op)
    vector<int> ts(opts, opts + n_opts);
    if (!HostMinValuesOK(d, hc, *R, ts)) return;
  }
  const int kct = d.key(kCapType), bspot = kct >= 0 ? d.bit(kct, "spot") : -1;
  const bool ncSpot = kct < 0 || !((R->present >> kct) & 1) || (bspot >= 0 ? Has(d, *R, kct, bspot) : ((R->compl_ >> kct) & 1));
  const bool s2s = allSpot && ncSpot;  // spot-to-spot: only behind the feature gate
  if (s2s && !cl.spot_to_spot) return;
  auto worst = [&](int t) {
    return tab ? tab->Worst(d, *R, types[t], tab->off[ci][t], s2s) : WorstLaunch(d, *R, types[t], s2s);
  };
  vector<int> kept;
  for (uint32_t i = 0; i < n_opts; i++)
    if (worst((int)opts[i]) < candPrice) kept.push_back((int)opts[i]);
  if (hasMin && !HostMinValuesOK(d, hc, *R, kept)) return;
  if (kept.empty()) return;
  if (multi_node) {  // filterOutSameType: the candidates' cheapest price per type name
    vector<std::pair<const string*, double>> prices;
    for (uint32_t c : cand) {
      const kp_cluster_node& n = cl.nodes[c];
      const HostType& it = cl.catalogs[n.catalog]->types[n.instance_type];
      double p = 0;
      if (cc ? !cc->priced[c] : !NodeCandidatePrice(it, labels[c], &p)) continue;
      if (cc) p = cc->price[c];
      bool found = false;
      for (auto& e : prices)
        if (*e.first == it.name) {
          e.second = std::min(e.second, p);
          found = true;
        }
      if (!found) prices.push_back({&it.name, p});
    }
    double maxPrice = std::numeric_limits<double>::max();
    for (int t : kept)
      for (auto& e : prices)
        if (*e.first == types[t].name && e.second < maxPrice) maxPrice = e.second;
    vector<int> k2;
    for (int t : kept)
      if (worst(t) < maxPrice) k2.push_back(t);
    if (hasMin && !HostMinValuesOK(d, hc, *R, k2)) return;
    kept.swap(k2);
    if (kept.empty()) return;
  }
  if (s2s && cand.size() == 1) {
    if (kept.size() < 15) return;
    kept.resize(std::min<size_t>(kept.size(), hasMin ? 100 : 15));
  }
  double best = std::numeric_limits<double>::max();
  for (int t : kept) best = std::min(best, worst(t));
  r.decision = KP_DECISION_REPLACE;
  r.nodepool = nodepool;
  r.replacement_price = best;
  r.savings = candPrice - best;
  r.n_options = (uint32_t)kept.size();
}

// FinalizeScheduling: a NodeClaim holding reservations launches only into them (reservation-id In {held ids})
static void ApplyHeld(const SolveBase& B, uint64_t held, KReqs& q) {
  if (!held) return;
  const Dict& d = B.d;
  const int k = d.key(kResID);
  for (int wi = 0; wi < nwords(d, k); wi++) q.vals[kw(d, k, wi)] = 0;
  for (uint64_t m = held; m; m &= m - 1) {
    const int bit = B.classes[__builtin_ctzll(m)].rid_bit;
    q.vals[bit / 64] |= 1ull << (bit % 64);
  }
  q.present |= 1ull << k;
  q.compl_ &= ~(1ull << k);
}

// One subset's SimulateScheduling as its own Solve: compiled on the host from the subset's inputs (the path for
// subsets the batch cannot take, and the whole path with KP_GENERAL_BATCH=0).
static int32_t GeneralSimOne(kp_cluster_plan* plan, const vector<uint32_t>& cand, const vector<std::map<string, string>>& labels,
                             int32_t multi_node, SimOut& r, uint64_t* counters, double* dev_ms, kp_cancel* cancel) {
  kp_ctx* ctx = plan->ctx;
  const kp_cluster& cl = plan->general->cl;
  const int N = (int)cl.n_nodes;
  vector<char> inS(N, 0);
  for (uint32_t c : cand) inS[c] = 1;
  vector<kp_existing_node> ex;
  vector<int> exNode;
  for (int i = 0; i < N; i++)
    if (!inS[i] && !cl.nodes[i].deleting) {
      ex.push_back(cl.nodes[i].node);
      exNode.push_back(i);
    }
  vector<kp_pod> pods;
  vector<int> kind;  // 0 candidate pod, 1 deleting-node pod, 2 pending
  for (uint32_t j = 0; j < cl.n_pending; j++) {
    if (cl.pending_pods[j] >= cl.n_pods) return fail(KP_E_INVAL, "pending pod %u", cl.pending_pods[j]);
    pods.push_back(cl.pods[cl.pending_pods[j]]);
    kind.push_back(2);
  }
  for (int i = 0; i < N; i++)
    if (cl.nodes[i].deleting)
      for (uint32_t j = 0; j < cl.nodes[i].n_pods; j++) {
        pods.push_back(cl.pods[cl.nodes[i].pods[j]]);
        kind.push_back(1);
      }
  for (uint32_t c : cand)
    for (uint32_t j = 0; j < cl.nodes[c].n_pods; j++) {
      pods.push_back(cl.pods[cl.nodes[c].pods[j]]);
      kind.push_back(0);
    }
  vector<kp_bound_pod> bound;
  for (size_t e = 0; e < exNode.size(); e++) {
    const kp_cluster_node& n = cl.nodes[exNode[e]];
    for (uint32_t j = 0; j < n.n_pods; j++) {
      const uint32_t p = n.pods[j];
      if (p >= cl.n_pods || cl.pods[p].shape >= cl.n_shapes) return fail(KP_E_INVAL, "node %d: pod %u", exNode[e], p);
      const kp_pod_shape& sh = cl.shapes[cl.pods[p].shape];
      bound.push_back({sh.namespace_, sh.labels, sh.n_labels, (uint32_t)e, sh.required_anti_affinity,
                       sh.n_required_anti_affinity, 0});
    }
  }
  r.n_pods = (uint32_t)pods.size();
  kp_solve_in in;
  memset(&in, 0, sizeof in);
  in.catalogs = cl.catalogs;
  in.n_catalogs = cl.n_catalogs;
  in.n_nodepools = cl.n_nodepools;
  in.nodepools = cl.nodepools;
  in.existing = ex.data();
  in.n_existing = (uint32_t)ex.size();
  in.n_shapes = cl.n_shapes;
  in.shapes = cl.shapes;
  in.pods = pods.data();
  in.n_pods = (uint32_t)pods.size();
  in.max_instance_types = 100;
  in.bound_pods = bound.data();
  in.n_bound_pods = (uint32_t)bound.size();
  in.namespaces = cl.namespaces;
  in.n_namespaces = cl.n_namespaces;
  in.reserved_offering_mode = KP_RESERVED_STRICT;  // SimulateScheduling: NewScheduler(..., DisableReservedCapacityFallback)
  kp_solve_plan* sp = nullptr;
  int32_t rc = SolvePrepare(ctx, &in, nullptr, &sp);
  if (rc) return rc;
  std::unique_ptr<kp_solve_plan, void (*)(kp_solve_plan*)> spg(sp, kp_solve_plan_destroy);
  kp_solve_result* res = nullptr;
  rc = kp_solve_run_cancellable(sp, cancel, &res);
  if (rc) return rc;
  std::unique_ptr<kp_solve_result, void (*)(kp_solve_result*)> rg(res, kp_result_destroy);
  counters[0] += res->stats.attempts;
  counters[1] += res->stats.bytes_algorithmic;
  counters[2] += res->stats.pops;
  *dev_ms += res->stats.device_ms;
  // AllNonPendingPodsScheduled; a candidate pod on an uninitialized node is an error (deleting-node pods exempt)
  bool all = true;
  for (size_t p = 0; p < pods.size() && all; p++) {
    const int32_t pl = res->placement[p];
    if (kind[p] == 2) continue;
    if (pl == -1) all = false;
    else if (kind[p] == 0 && pl <= -2 && !ex[(size_t)(-2 - pl)].initialized) all = false;
  }
  const int n_nc = (int)res->ncs.size();
  // (kp_solve_run already applied the held reservations and the minValues truncation check to NodeClaim 0)
  GeneralDecide(cl, labels, cand, *sp->cp->B, all, n_nc, n_nc ? &res->fin[0] : nullptr, n_nc ? res->nc_cat[0] : 0,
                n_nc ? res->ncs[0].nodepool : 0, n_nc ? res->ncs[0].options.data() : nullptr,
                n_nc ? (uint32_t)res->ncs[0].options.size() : 0, multi_node, r);
  return KP_OK;
}

// ---- batched general simulations ------------------------------------------------------------------------------
// Compiling each subset's Solve on the host walks every node and every bound pod (~18 ms per subset at 2000 nodes).
// Instead the cluster is compiled once as the superset Solve - every node not being deleted is an existing node,
// every pod a simulation can queue (pending, deleting nodes', every node's) is in its pod list - with each node's
// contribution to the topology state recorded (Compiled::track_nodes). A subset's Solve is that Solve with:
//   * the subset's nodes excluded from placement (ex_static_ok 0) - the other nodes keep their relative order;
//   * its queue: the pending and deleting-node pods plus the subset's pods, in the superset's queue order (the same
//     keys: shape rank, creation, UID);
//   * the bound pods on its nodes removed from the topology counts and registered domains (Topology.countDomains
//     over the remaining nodes), hostname rows' "some domain has a count" recomputed;
//   * the spread groups' liveness recomputed from the shapes it queues (NewTopology creates the groups of queued
//     pods), and hostname groups that stop being live at creation get their unregistered nodes (255) back.
// Subsets whose removal would make an inverse anti-affinity group vanish take the per-subset compile. Every
// simulation of a batch is one workgroup of one solve_kernel launch (its own arena: mutable state + scratch).
// Host memory the device copies read from / write into while the host prepares the next launch (pinned: an async
// copy from pageable memory would stage synchronously), grown geometrically.
struct PinnedBuf {
  void* p = nullptr;
  size_t n = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t reserve(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    const size_t want = std::max(bytes, (size_t)(1.5 * (double)bytes));
    const hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) n = want;
    else p = nullptr;
    return e;
  }
  uint8_t* at(size_t off) const { return (uint8_t*)p + off; }
};

// One launch slot of the general batch: device arenas + argument blocks, the pinned host copies its launch reads
// (overlays, arguments) and writes (results), and the event that marks its results landed.
struct GenSlot {
  DevBuf arenas, args;
  size_t arenas_bytes = 0, args_bytes = 0;
  PinnedBuf up, down;
  hipEvent_t done = nullptr, t0 = nullptr, t1 = nullptr;  // results landed; the launch's kernels (timing)
  hipEvent_t uploaded = nullptr;                            // the launch's overlays and arguments on the device
  int n = 0;
  size_t b0 = 0;
  vector<vector<int32_t>> queues;
  ~GenSlot() {
    for (hipEvent_t e : {done, t0, t1, uploaded})
      if (e) (void)hipEventDestroy(e);
  }
};
// the batch's copy streams: uploads (the next launch's overlays) and downloads (the last launch's results) overlap the
// kernels instead of queueing between them; and one kernel stream per launch slot, so that a launch's batch_init and
// first workgroups fill the CUs the previous launch's last simulations leave idle (the slots share only read-only data)
struct CopyStreams {
  hipStream_t up = nullptr, down = nullptr, k[2] = {nullptr, nullptr};
  ~CopyStreams() {
    for (hipStream_t x : {up, down, k[0], k[1]})
      if (x) (void)hipStreamDestroy(x);
  }
};

struct GeneralBatch {
  std::unique_ptr<Compiled> C;
  size_t ulist_total = 0;  // entries of the per-shape-level usable lists (the batched existing-node memo's size)
  uint64_t base_version = 0;
  vector<int32_t> node_input;   // cluster node -> existing input index of the superset (-1: being deleted)
  vector<int32_t> node_sorted;  // cluster node -> position in the Solve's existing order (-1)
  vector<int32_t> pos_node;     // existing position -> cluster node
  vector<int32_t> pod_qpos;     // superset pod -> queue position
  vector<int32_t> pod_shape;    // superset pod -> shape
  vector<int32_t> base_pods;    // superset pods every simulation queues (pending, deleting nodes'), queue order
  vector<uint8_t> pod_kind;     // superset pod -> 2 pending, 1 deleting node's, 0 a node's
  vector<vector<int32_t>> node_pods;  // cluster node -> its superset pods
  vector<uint8_t> ex_static;
  vector<int32_t> regcnt;       // [G * 64] existing nodes registering each (group, ordinal)
  vector<int32_t> live0;        // [G] liveness with only the base pods queued
  OfferTab offers;              // the decisions' offering bits (the superset's dictionary)
  CandCache cands;              // the candidates' prices
  uint32_t rmask = 0;
  int res_mode = 0, opt_stride = 100, tf_words = 0;
  bool tfeas_on = false;
  SolveOffs so;                 // shared-region offsets
  DevBuf shared;
  // per arena size (Pc): the layout, the host template of [0, mut_end) and the device copy of [common, mut_end)
  int Pc = 0;
  SolveOffs o;
  size_t stride = 0;
  vector<uint8_t> tmpl;
  DevBuf pristine;
  GenSlot slot[2];  // two launch slots (GeneralBatchRun)
  CopyStreams cs;
};

// The superset Solve of a cluster (kp_cluster_plan: general). KP_E_UNSUPPORTED: the batch cannot take this cluster
// (the caller keeps the per-subset compile).
static int32_t GeneralBatchBuild(kp_cluster_plan* plan, std::shared_ptr<GeneralBatch>& out) {
  kp_ctx* ctx = plan->ctx;
  const kp_cluster& cl = plan->general->cl;
  const int N = (int)cl.n_nodes;
  PhaseTimer pt;
  auto gb = std::make_shared<GeneralBatch>();
  vector<kp_existing_node> ex;
  vector<kp_pod> pods;
  vector<kp_bound_pod> bound;
  gb->node_input.assign(N, -1);
  gb->node_pods.assign(N, {});
  for (uint32_t j = 0; j < cl.n_pending; j++) {
    if (cl.pending_pods[j] >= cl.n_pods) return fail(KP_E_INVAL, "pending pod %u", cl.pending_pods[j]);
    pods.push_back(cl.pods[cl.pending_pods[j]]);
    gb->pod_kind.push_back(2);
  }
  for (int i = 0; i < N; i++)
    if (cl.nodes[i].deleting)
      for (uint32_t j = 0; j < cl.nodes[i].n_pods; j++) {
        pods.push_back(cl.pods[cl.nodes[i].pods[j]]);
        gb->pod_kind.push_back(1);
      }
  const int n_base = (int)pods.size();
  for (int i = 0; i < N; i++) {
    if (cl.nodes[i].deleting) continue;
    const uint32_t e = (uint32_t)ex.size();
    gb->node_input[i] = (int32_t)e;
    ex.push_back(cl.nodes[i].node);
    for (uint32_t j = 0; j < cl.nodes[i].n_pods; j++) {
      const uint32_t p = cl.nodes[i].pods[j];
      if (p >= cl.n_pods || cl.pods[p].shape >= cl.n_shapes) return fail(KP_E_INVAL, "node %d: pod %u", i, p);
      const kp_pod_shape& sh = cl.shapes[cl.pods[p].shape];
      bound.push_back({sh.namespace_, sh.labels, sh.n_labels, e, sh.required_anti_affinity, sh.n_required_anti_affinity, 0});
      gb->node_pods[i].push_back((int32_t)pods.size());
      pods.push_back(cl.pods[p]);
      gb->pod_kind.push_back(0);
    }
  }
  {  // queue ties broken by pod index would order differently per subset: only distinct (creation, UID) keys
    vector<std::pair<int64_t, uint64_t>> keys;
    for (auto& p : pods) keys.push_back({p.creation_unix, p.uid_key});
    std::sort(keys.begin(), keys.end());
    if (std::adjacent_find(keys.begin(), keys.end()) != keys.end())
      return fail(KP_E_UNSUPPORTED, "pods with equal (creation, UID) keys");
  }
  kp_solve_in in;
  memset(&in, 0, sizeof in);
  in.catalogs = cl.catalogs;
  in.n_catalogs = cl.n_catalogs;
  in.n_nodepools = cl.n_nodepools;
  in.nodepools = cl.nodepools;
  in.existing = ex.data();
  in.n_existing = (uint32_t)ex.size();
  in.n_shapes = cl.n_shapes;
  in.shapes = cl.shapes;
  in.pods = pods.data();
  in.n_pods = (uint32_t)pods.size();
  in.max_instance_types = 100;
  in.bound_pods = bound.data();
  in.n_bound_pods = (uint32_t)bound.size();
  in.namespaces = cl.namespaces;
  in.n_namespaces = cl.n_namespaces;
  in.reserved_offering_mode = KP_RESERVED_STRICT;
  pt.lap("general: inputs");
  gb->C = std::make_unique<Compiled>();
  Compiled& C = *gb->C;
  C.track_nodes = true;
  int32_t rc = CompileSolve(&in, C, ctx);
  if (rc) return rc;
  pt.lap("general: superset compile");
  if (!C.track_nodes) return fail(KP_E_INVAL, "superset compile lost its node tracking");
  rc = EnsureBaseOnDevice(ctx, *C.B);
  if (rc) return rc;
  gb->base_version = C.B->version;
  const int E = (int)C.ex_input.size(), G = C.G, P = (int)pods.size();
  gb->node_sorted.assign(N, -1);
  gb->pos_node.assign(E, -1);
  vector<int32_t> input_node(E, -1);
  for (int i = 0; i < N; i++)
    if (gb->node_input[i] >= 0) input_node[gb->node_input[i]] = i;
  for (int e = 0; e < E; e++) {
    gb->pos_node[e] = input_node[C.ex_input[e]];
    gb->node_sorted[gb->pos_node[e]] = e;
  }
  gb->pod_qpos.assign(P, 0);
  gb->pod_shape = C.pod_shape;
  for (int q = 0; q < P; q++) gb->pod_qpos[C.queue[q]] = q;
  for (int q = 0; q < P; q++)
    if (C.queue[q] < n_base) gb->base_pods.push_back(C.queue[q]);
  if (G) {
    if (C.node_cnt.size() != (size_t)E || C.tg_spread.size() != (size_t)G || C.shape_l0.size() != cl.n_shapes)
      return fail(KP_E_INVAL, "superset topology tracking incomplete");
    gb->regcnt.assign((size_t)G * 64, 0);
    for (auto& v : C.node_reg)
      for (int32_t x : v) gb->regcnt[x]++;
    gb->live0.assign(G, 0);
    for (int g = 0; g < G; g++) gb->live0[g] = C.tg_live[g] && !C.tg_spread[g];
    vector<char> seen(cl.n_shapes, 0);
    for (int p : gb->base_pods) {
      const int s = C.pod_shape[p];
      if (seen[s]) continue;
      seen[s] = 1;
      for (int32_t g : C.shape_l0[s]) gb->live0[g] = 1;
    }
  }
  pt.lap("general: tracking");
  gb->rmask = RequestedResources(C);
  gb->ex_static = ExStatic(C, gb->rmask);
  gb->offers.Build(C.B->d, cl);
  pt.lap("general: offers");
  {  // (the candidate prices read the capacity-type, zone, zone-id and reservation labels only)
    vector<std::map<string, string>> labels(N);
    for (int i = 0; i < N; i++)
      for (uint32_t j = 0; j < cl.nodes[i].node.n_labels; j++) {
        const kp_label& l = cl.nodes[i].node.labels[j];
        string k = Normalize(l.key ? l.key : "");
        if (k == kCapType || k == kZone || k == kZoneID || k == kResID || k == kResType)
          labels[i][std::move(k)] = l.value ? l.value : "";
      }
    gb->cands.Build(cl, labels);
  }
  pt.lap("general: candidates");
  gb->res_mode = !C.B->res_cls ? 0 : 2;
  gb->opt_stride = 100;
  // the shared region: read-only data of every simulation + the template-options table
  Blob blob;
  PutShared(blob, C, gb->so);
  pt.lap("general: shared blob");
  {  // per shape-level, the positions that can ever take one of its pods (DeviceArgs::ex_ulist): the kernel's
     // count-independent checks on the pristine state
    const int E = (int)C.ex_input.size(), SLn = (int)C.shape_reqs.size();
    vector<int32_t> sl_shape(SLn, 0), off(SLn + 1, 0), list, uidx((size_t)SLn * std::max(E, 1), 0);
    for (size_t s = 0; s < C.shape_level_base.size(); s++)
      for (int l = 0; l < C.shape_nlevels[s]; l++) sl_shape[C.shape_level_base[s] + l] = (int32_t)s;
    for (int sl = 0; sl < SLn; sl++) {
      off[sl] = (int32_t)list.size();
      const int s = sl_shape[sl];
      const int64_t* pq = &C.shape_requests[(size_t)s * KP_NRES];
      const uint64_t tol = C.shape_tolerates[sl], hpc = C.hp_any ? C.shape_hp_conf[s] : 0;
      for (int e = 0; e < E; e++) {
        uidx[(size_t)sl * E + e] = (int32_t)(list.size() - off[sl]);
        bool ok = gb->ex_static[e] && ((tol >> C.ex_taintset[e]) & 1) && !(hpc && (C.ex_hp[e] & hpc));
        for (uint32_t m = gb->rmask; m && ok; m &= m - 1) {
          const int r = __builtin_ctz(m);
          ok = C.ex_available[(size_t)e * KP_NRES + r] - C.ex_requests[(size_t)e * KP_NRES + r] >= pq[r];
        }
        if (ok) list.push_back(e);
      }
    }
    off[SLn] = (int32_t)list.size();
    gb->ulist_total = list.size();  // (the batched arenas' existing-node memo: one entry per list entry)
    if (list.empty()) list.push_back(0);
    gb->so.exul = blob.put(list);
    gb->so.exuo = blob.put(off);
    gb->so.exui = blob.put(uidx);
  }
  pt.lap("general: usable lists");
  const size_t host_bytes = blob.host.size();
  const int NT = (int)C.B->tmpl_reqs.size(), SLi = (int)C.shape_reqs.size();
  gb->tfeas_on = NT > 0 && SLi > 0 && ctx->ov.template_table == 0;
  gb->tf_words = C.B->TW + KP_NRES / 2 + 1;
  gb->so.tfeas = blob.reserve_dev(gb->tfeas_on ? (size_t)SLi * NT * gb->tf_words * sizeof(uint64_t) : 8);
  HIPCHK(gb->shared.alloc(blob.total()));
  uint8_t* sh = (uint8_t*)gb->shared.p;
  HIPCHK(hipMemcpyAsync(sh, blob.host.data(), host_bytes, hipMemcpyHostToDevice, ctx->stream));
  if (gb->tfeas_on) {
    SolveArgs a;
    BindSolve(a, C, gb->so, sh, sh, 0, 1, gb->rmask, gb->res_mode);
    HIPCHK(launch_tmpl_feas(TfeasOf(a, sh, gb->so, SLi, gb->tf_words), ctx->stream));
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));
  pt.lap("general: upload + table");
  out = gb;
  return KP_OK;
}

// The arena layout for simulations of up to Pc pods: host template + the device copy of the common mutable part.
static int32_t GeneralBatchLayout(kp_ctx* ctx, GeneralBatch& gb, int Pc) {
  if (gb.Pc == Pc) return KP_OK;
  const Compiled& C = *gb.C;
  SolveOffs o = gb.so;
  Blob blob;
  const vector<int32_t> zeros(Pc, 0);
  PutArena(blob, C, zeros, zeros, Pc, gb.ex_static, gb.rmask, o);
  ReserveArenaDev(blob, C, Pc, gb.opt_stride, std::min(SortCapacity(C.ov), Pc), false, o, gb.ulist_total);
  gb.tmpl.assign(blob.host.begin(), blob.host.begin() + o.mut_end);
  gb.stride = (o.arena_end + 255) & ~(size_t)255;
  HIPCHK(gb.pristine.alloc(o.mut_end - o.common + 16));
  HIPCHK(hipMemcpyAsync(gb.pristine.p, gb.tmpl.data() + o.common, o.mut_end - o.common, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  gb.o = o;
  gb.Pc = Pc;
  return KP_OK;
}

// One simulation's per-subset inputs: its queue (superset pods) and the patch of [0, common) of its arena. Returns 1
// when the batch cannot take the subset (an inverse anti-affinity group would vanish).
struct GenScratch {
  vector<int32_t> inv, hdec, regdec, touched;
  vector<char> shape_seen;
};
// The host work of a batched launch is per simulation (the overlays before it, the decisions after it): split over up
// to kMaxHostThreads threads, f(begin, end, thread index). Workers never call fail() (its message is thread-local).
constexpr int kMaxHostThreads = 16;
extern "C++" template <class F>
static void ParallelFor(int n, F f) {
  static const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  const int T = std::max(1, std::min(std::min(hw, kMaxHostThreads), n / 128));
  if (T <= 1) {
    f(0, n, 0);
    return;
  }
  vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; t++) th.emplace_back(f, (int)((int64_t)n * t / T), (int)((int64_t)n * (t + 1) / T), t);
  f(0, (int)((int64_t)n / T), 0);
  for (auto& x : th) x.join();
}
static int GeneralPatch(const GeneralBatch& gb, const kp_cluster& cl, const vector<uint32_t>& cand, GenScratch& s,
                        vector<int32_t>& queue, uint8_t* patch) {
  const Compiled& C = *gb.C;
  const int G = C.G, E = (int)C.ex_input.size();
  if (G) {  // an inverse group whose every owner sits on the subset's nodes does not exist in its Solve
    s.inv.assign(G, 0);
    bool vanish = false;
    for (uint32_t c : cand)
      for (int32_t g : C.node_inv[gb.node_input[c]])
        if (++s.inv[g] == C.tg_inv_total[g]) vanish = true;
    if (vanish) return 1;
  }
  queue = gb.base_pods;
  const size_t nb = queue.size();
  for (uint32_t c : cand) queue.insert(queue.end(), gb.node_pods[c].begin(), gb.node_pods[c].end());
  auto byq = [&](int32_t x, int32_t y) { return gb.pod_qpos[x] < gb.pod_qpos[y]; };
  std::sort(queue.begin() + nb, queue.end(), byq);
  std::inplace_merge(queue.begin(), queue.begin() + nb, queue.end(), byq);
  const SolveOffs& o = gb.o;
  memcpy(patch, gb.tmpl.data(), o.common);
  int32_t* ps = (int32_t*)(patch + o.pod_shape);
  int32_t* qu = (int32_t*)(patch + o.queue);
  for (size_t i = 0; i < queue.size(); i++) {
    ps[i] = gb.pod_shape[queue[i]];
    qu[i] = (int32_t)i;
  }
  uint8_t* exso = patch + o.exso;
  for (uint32_t c : cand) exso[gb.node_sorted[c]] = 0;
  if (!G) return 0;
  int32_t* cnt = (int32_t*)(patch + o.tgc);
  int32_t* live = (int32_t*)(patch + o.tglv);
  uint64_t* reg = (uint64_t*)(patch + o.tgreg);
  uint8_t* hcx = patch + o.hcx;
  s.regdec.resize((size_t)G * 64);
  s.hdec.assign(G, 0);
  s.touched.clear();
  for (uint32_t c : cand) {
    const int e = gb.node_input[c];
    for (int32_t x : C.node_cnt[e]) cnt[x]--;
    for (int32_t x : C.node_reg[e]) {
      if (s.regdec[x]++ == 0) s.touched.push_back(x);
    }
    for (int32_t g : C.node_hrec[e]) s.hdec[g]++;
  }
  for (int32_t x : s.touched) {
    const int g = x / 64, ord = x % 64;
    if (s.regdec[x] == gb.regcnt[x] && !((C.tg_reg_static[g] >> ord) & 1)) reg[g] &= ~(1ull << ord);
    s.regdec[x] = 0;
  }
  for (int g = 0; g < G; g++)
    if (s.hdec[g] && s.hdec[g] == C.tg_hrec_total[g]) reg[g] &= ~1ull;  // hostname row: no domain has a count
  // liveness: the base pods' shapes, then the subset's
  for (int g = 0; g < G; g++) live[g] = gb.live0[g];
  s.shape_seen.assign(cl.n_shapes, 0);
  for (size_t i = nb; i < queue.size(); i++) {
    const int sh = gb.pod_shape[queue[i]];
    if (s.shape_seen[sh]) continue;
    s.shape_seen[sh] = 1;
    for (int32_t g : C.shape_l0[sh]) live[g] = 1;
  }
  for (int g = 0; g < G; g++)  // a hostname spread group created not live: its unregistered nodes hold 255
    if (C.tg_live[g] && !live[g] && C.tg_spread[g] && C.tg_row[g] >= 0)
      for (int32_t pos : C.tg_unreg[g]) hcx[(size_t)C.tg_row[g] * E + pos] = 255;
  return 0;
}

// Runs the batchable subsets `idx` (their candidate lists in cands) as batched Solves; outs[idx[i]] get the decisions.
static int32_t GeneralBatchRun(kp_cluster_plan* plan, GeneralBatch& gb, const vector<vector<uint32_t>>& cands,
                               const vector<int>& idx, const vector<std::map<string, string>>& labels, int32_t multi_node,
                               vector<SimOut>& outs, uint64_t* counters, double* dev_ms, double* host_ms,
                               kp_cancel* cancel, uint64_t* n_launches) {
  kp_ctx* ctx = plan->ctx;
  const kp_cluster& cl = plan->general->cl;
  const Compiled& C = *gb.C;
  hipStream_t st = ctx->stream;
  // kp_cancel: solve_kernel polls the flag (every ~1,024 pops of each simulation) and the host reads it before each
  // launch; any early return (cancellation, an error) first drains the launches this call queued
  const int32_t* dcancel = nullptr;
  if (cancel) {
    void* dp = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dp, cancel->flag, 0));
    dcancel = (const int32_t*)dp;
  }
  struct Drain {
    hipStream_t s;
    ~Drain() { (void)hipStreamSynchronize(s); }
  } drain{st};
  // the arena size: every simulation of the batch fits (rounded up, so that nearby batches share a layout)
  size_t max_pods = 1;
  vector<size_t> len(cands.size(), 0);
  for (int i : idx) {
    size_t n = gb.base_pods.size();
    for (uint32_t c : cands[i]) n += gb.node_pods[c].size();
    len[i] = n;
    max_pods = std::max(max_pods, n);
  }
  int Pc = 64;
  while ((size_t)Pc < max_pods) Pc *= 2;
  if (int32_t rc = GeneralBatchLayout(ctx, gb, Pc)) return rc;
  const SolveOffs& o = gb.o;
  const size_t patch_bytes = o.common;
  // simulations per launch: two launch slots (the host prepares one while the device runs the other), each at most
  // an eighth of the free device memory in arenas and 4096 simulations (one Solve workgroup per CU runs at a time;
  // the rest queue behind it)
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = (size_t)8 << 30;
  const size_t held_b = gb.slot[0].arenas_bytes + gb.slot[1].arenas_bytes;
  const size_t budget = std::max<size_t>((free_b + held_b) / 8, (size_t)1 << 30);
  size_t per_launch = std::max<size_t>(1, std::min<size_t>(4096, budget / gb.stride));
  if (idx.size() > per_launch && idx.size() < 2 * per_launch) per_launch = (idx.size() + 1) / 2;  // two even launches
  // longest simulations first (queue length: pending + the candidates' pods): they start on the first CUs instead
  // of trailing the launch
  vector<int> order(idx);
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return len[x] > len[y]; });
  if (ctx->ov.host_timing)
    fprintf(stderr, "[kp general] arena stride %.2f MB, %zu simulations per launch, Pc %d; batch_init per simulation: copy %zu B, "
            "fills stats %zu npods %zu place %zu ver %zu fail %zu hcnc %zu B\n", gb.stride / 1e6, per_launch, Pc,
            gb.o.exr - gb.o.common - (__builtin_popcount(gb.rmask) <= 4 ? gb.o.exroom - gb.o.exrq : 0),
            sizeof(uint64_t) * KP_SOLVE_STATS, sizeof(int32_t) * (size_t)Pc, sizeof(int32_t) * (size_t)Pc,
            gb.o.ver_end - gb.o.ver0, gb.o.fail_end - gb.o.fail0, gb.o.n_hcnc);
  const int sort_cap = std::min(SortCapacity(C.ov), Pc);
  const size_t dyn = std::max<size_t>((size_t)2 * sort_cap * sizeof(int32_t), o.chk_on ? CHK_LDS_BYTES : 0);
  vector<GenScratch> scratches(kMaxHostThreads);
  vector<SolveArgs> sargs;
  vector<FinalizeArgs> fargs;
  // per-launch result layout in the slot's pinned download buffer
  const size_t r_stats = 0, r_place = r_stats + sizeof(uint64_t) * KP_SOLVE_STATS * per_launch;
  const size_t r_nct = r_place + sizeof(int32_t) * (size_t)Pc * per_launch;
  const size_t r_nopt = r_nct + sizeof(int32_t) * per_launch;
  const size_t r_opts = r_nopt + sizeof(uint32_t) * per_launch;
  const size_t r_fin = (r_opts + sizeof(uint32_t) * (size_t)gb.opt_stride * per_launch + 63) & ~(size_t)63;
  const size_t r_held = r_fin + sizeof(KReqs) * per_launch;
  const size_t r_end = r_held + sizeof(uint64_t) * per_launch;
  const size_t u_args = (patch_bytes * per_launch + 255) & ~(size_t)255;
  const size_t u_fargs = u_args + ((sizeof(SolveArgs) * per_launch + 255) & ~(size_t)255);
  const size_t u_end = u_fargs + sizeof(FinalizeArgs) * per_launch;

  // the host decisions of a finished launch (its results in the slot's download buffer)
  auto decide = [&](GenSlot& sl) -> int32_t {
    HIPCHK(hipEventSynchronize(sl.done));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, sl.t0, sl.t1));
    *dev_ms += ms;
    const auto th1 = std::chrono::steady_clock::now();
    const int n = sl.n;
    const size_t b0 = sl.b0;
    const uint64_t* stats = reinterpret_cast<uint64_t*>(sl.down.at(r_stats));
    const int32_t* place = reinterpret_cast<int32_t*>(sl.down.at(r_place));
    const int32_t* nct = reinterpret_cast<int32_t*>(sl.down.at(r_nct));
    const uint32_t* nopt = reinterpret_cast<uint32_t*>(sl.down.at(r_nopt));
    uint32_t* opts = reinterpret_cast<uint32_t*>(sl.down.at(r_opts));
    const KReqs* fin = reinterpret_cast<KReqs*>(sl.down.at(r_fin));
    const uint64_t* held = reinterpret_cast<uint64_t*>(sl.down.at(r_held));
    const vector<vector<int32_t>>& queues = sl.queues;
    std::atomic<int> bad_runaway{-1}, cancelled{0};
    uint64_t tcount[kMaxHostThreads][3] = {}, tphase[kMaxHostThreads][8] = {};
    ParallelFor(n, [&](int j_lo, int j_hi, int t) {
    for (int j = j_lo; j < j_hi; j++) {
      const int i = order[b0 + j];
      const uint64_t* sj = &stats[(size_t)j * KP_SOLVE_STATS];
      if (sj[7]) {
        bad_runaway = i;
        return;
      }
      if (sj[46]) {
        cancelled = 1;
        return;
      }
      tcount[t][0] += sj[0];
      tcount[t][1] += sj[1];
      tcount[t][2] += sj[2];
      for (int k = 0; k < 8; k++) tphase[t][k] += sj[8 + k];  // (zero unless kp_overrides.timing)
      const int n_nc = (int)sj[3];
      const vector<int32_t>& q = queues[j];
      SimOut& r = outs[i];
      r.n_pods = (uint32_t)q.size();
      // AllNonPendingPodsScheduled; a candidate pod on an uninitialized node is an error (deleting-node pods exempt)
      bool all = true;
      for (size_t p = 0; p < q.size() && all; p++) {
        const uint8_t kind = gb.pod_kind[q[p]];
        const int32_t pl = place[(size_t)j * Pc + p];
        if (kind == 2) continue;
        if (pl == -1) all = false;
        else if (kind == 0 && pl <= -2 && !cl.nodes[gb.pos_node[-2 - pl]].node.initialized) all = false;
      }
      KReqs R = fin[j];
      int ci = 0;
      uint32_t np = 0;
      if (n_nc == 1) {
        if (gb.res_mode) ApplyHeld(*C.B, held[j], R);
        ci = C.B->tmpl_catalog[nct[j]];
        np = (uint32_t)C.B->tmpl_nodepool[nct[j]];
      }
      GeneralDecide(cl, labels, cands[i], *C.B, all, n_nc, &R, ci, np, &opts[(size_t)j * gb.opt_stride],
                    n_nc == 1 ? nopt[j] : 0, multi_node, r, &gb.offers, &gb.cands);
    }
    });
    for (int t = 0; t < kMaxHostThreads; t++) {
      for (int k = 0; k < 3; k++) counters[k] += tcount[t][k];
      for (int k = 0; k < 8; k++) plan->general_phase[k] += tphase[t][k];
    }
    if (bad_runaway >= 0)
      return fail(KP_E_DEVICE, "solve_kernel exceeded its Queue.Pop bound in simulation %d: aborted", bad_runaway.load());
    if (cancelled) return fail(KP_E_CANCELED, "consolidation simulations cancelled (kp_cancel_set)");
    host_ms[1] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th1).count();
    return KP_OK;
  };

  GenSlot* slots = gb.slot;
  for (int k = 0; k < 2; k++)
    if (!slots[k].done) {
      HIPCHK(hipEventCreateWithFlags(&slots[k].done, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&slots[k].uploaded, hipEventDisableTiming));
      HIPCHK(hipEventCreate(&slots[k].t0));
      HIPCHK(hipEventCreate(&slots[k].t1));
    }
  if (!gb.cs.up) {
    HIPCHK(hipStreamCreateWithFlags(&gb.cs.up, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&gb.cs.down, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&gb.cs.k[0], hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&gb.cs.k[1], hipStreamNonBlocking));
  }
  hipStream_t up = gb.cs.up, dn = gb.cs.down;
  struct DrainCopies {  // (early returns: nothing left in flight on the copy or kernel streams either)
    hipStream_t u, d, k0, k1;
    ~DrainCopies() {
      for (hipStream_t x : {k0, k1, u, d}) (void)hipStreamSynchronize(x);
    }
  } drain_copies{up, dn, gb.cs.k[0], gb.cs.k[1]};
  int pending = -1;  // the slot whose launch is in flight and not yet decided
  int launch_no = 0;
  for (size_t b0 = 0; b0 < idx.size(); b0 += per_launch, launch_no++) {
    if (cancel && __atomic_load_n(cancel->flag, __ATOMIC_SEQ_CST))
      return fail(KP_E_CANCELED, "consolidation simulations cancelled (kp_cancel_set) after %zu of %zu", b0, idx.size());
    GenSlot& sl = slots[launch_no & 1];
    const auto th0 = std::chrono::steady_clock::now();
    const int n = (int)std::min(per_launch, idx.size() - b0);
    // arenas for this launch's n simulations, grown geometrically (a few subsets do not pin gigabytes on the plan);
    // when the device cannot hold them, this batch and the rest run one simulation at a time (GeneralSimOne)
    hipError_t ae = hipSuccess;
    if (sl.arenas_bytes < gb.stride * n) {
      const size_t sims = std::min(per_launch, std::max<size_t>((size_t)n, 2 * sl.arenas_bytes / gb.stride));
      ae = sl.arenas.alloc(gb.stride * sims);
      sl.arenas_bytes = ae == hipSuccess ? gb.stride * sims : 0;
    }
    const size_t args_need = (sizeof(SolveArgs) + sizeof(FinalizeArgs)) * (size_t)n + 512;
    if (ae == hipSuccess && sl.args_bytes < args_need) {
      ae = sl.args.alloc(args_need);
      sl.args_bytes = ae == hipSuccess ? args_need : 0;
    }
    if (ae == hipSuccess) ae = sl.up.reserve(u_end);
    if (ae == hipSuccess) ae = sl.down.reserve(r_end);
    if (ae != hipSuccess) {
      (void)hipGetLastError();
      if (pending >= 0) {
        if (int32_t rc = decide(slots[pending])) return rc;
        pending = -1;
      }
      for (size_t j = b0; j < idx.size(); j++)
        if (int32_t rc = GeneralSimOne(plan, cands[order[j]], labels, multi_node, outs[order[j]], counters, dev_ms, cancel)) return rc;
      break;
    }
    uint8_t* arenas = (uint8_t*)sl.arenas.p;
    uint8_t* sh = (uint8_t*)gb.shared.p;
    uint8_t* patches = reinterpret_cast<uint8_t*>(sl.up.at(0));
    sl.queues.resize(n);
    vector<vector<int32_t>>& queues = sl.queues;
    sargs.resize(n);
    fargs.resize(n);
    std::atomic<int> unbatchable{-1};
    const bool ht = ctx->ov.host_timing != 0;
    double tpatch[kMaxHostThreads] = {};  // (kp_overrides.host_timing: the overlays' own share)
    ParallelFor(n, [&](int j_lo, int j_hi, int t) {
    for (int j = j_lo; j < j_hi; j++) {
      const int i = order[b0 + j];
      const auto tp0 = ht ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
      if (GeneralPatch(gb, cl, cands[i], scratches[t], queues[j], patches + patch_bytes * j)) {
        unbatchable = i;
        return;
      }
      if (ht) tpatch[t] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();
      uint8_t* ar = arenas + gb.stride * j;
      SolveArgs& a = sargs[j];
      BindSolve(a, C, o, sh, ar, (int)queues[j].size(), Pc, gb.rmask, gb.res_mode);
      a.cancel = dcancel;
      a.stop_nc = 2;  // a second NodeClaim decides the simulation (no-op): the kernel ends its Solve there
      a.ex_reqs_ro = (const uint8_t*)gb.pristine.p + (o.exr - o.common);  // (the arena's copy is written on demand)
      a.ex_ulist = (const int32_t*)(sh + gb.so.exul);
      a.ex_ulist_off = (const int32_t*)(sh + gb.so.exuo);
      a.ex_uidx = (const int32_t*)(sh + gb.so.exui);
      if (gb.tfeas_on) {
        a.tfeas = (const uint64_t*)(sh + o.tfeas);
        a.tfeas_words = gb.tf_words;
      }
      FinalizeArgs& f = fargs[j];
      memset(&f, 0, sizeof f);
      f.dict = a.dict;
      f.cats = a.cats;
      f.vint = a.vint;
      f.nc_tmpl = a.nc_tmpl;
      f.tmpl_catalog = a.tmpl_catalog;
      f.nc_reqs = a.nc_reqs;
      f.nc_X = a.nc_X;
      f.max_types = 100;
      f.opt_stride = gb.opt_stride;
      f.out_options = (uint32_t*)(ar + o.opts);
      f.out_n_remaining = (uint32_t*)(ar + o.nrem);
      f.out_n_options = (uint32_t*)(ar + o.nopt);
      f.nc_held = a.res_mode ? a.nc_held : nullptr;
      f.solve_stats = a.stats;
    }
    });
    if (unbatchable >= 0) return fail(KP_E_INVAL, "subset %d: not batchable after the check", unbatchable.load());
    if (ht) {
      double tp = 0;
      for (double x : tpatch) tp += x;
      fprintf(stderr, "[kp general] launch %d: %d sims, patch %zu B each, GeneralPatch %.2f thread-ms, overlays %.2f ms\n",
              launch_no, n, patch_bytes, tp,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count());
    }
    memcpy(reinterpret_cast<uint8_t*>(sl.up.at(u_args)), sargs.data(), sizeof(SolveArgs) * n);
    memcpy(reinterpret_cast<uint8_t*>(sl.up.at(u_fargs)), fargs.data(), sizeof(FinalizeArgs) * n);
    SolveArgs* dargs = (SolveArgs*)sl.args.p;
    FinalizeArgs* dfargs = (FinalizeArgs*)((uint8_t*)sl.args.p + ((sizeof(SolveArgs) * n + 255) & ~(size_t)255));
    BatchInitArgs bi;
    memset(&bi, 0, sizeof bi);
    bi.base = arenas;
    bi.stride = gb.stride;
    bi.pristine = (const uint8_t*)gb.pristine.p;
    bi.dst_off = o.common;
    bi.n_copy = (o.exr - o.common + 15) & ~(size_t)15;  // not the existing nodes' requirements: copy-on-write
    if (__builtin_popcount(gb.rmask) <= 4) {
      // the existing nodes' request rows are read only for a fifth requested resource and beyond (the first four are
      // their headroom rows); with four or fewer a commit's read-modify-write leaves the unread values unread
      bi.skip_off = o.exrq - o.common;
      bi.skip_len = (o.exroom - o.exrq) & ~(size_t)15;
    }
    auto fill = [&](size_t off, size_t len, uint32_t byte) {
      bi.fill_off[bi.n_fill] = off;
      bi.fill_len[bi.n_fill] = (len + 15) & ~(size_t)15;
      bi.fill_byte[bi.n_fill] = byte;
      bi.n_fill++;
    };
    fill(o.stats, sizeof(uint64_t) * KP_SOLVE_STATS, 0);
    fill(o.npods, sizeof(int32_t) * Pc, 0);
    fill(o.place, sizeof(int32_t) * Pc, 0xFF);
    fill(o.ver0, o.ver_end - o.ver0, 0);
    fill(o.fail0, o.fail_end - o.fail0, 0xFF);
    if (o.n_hcnc) fill(o.hcnc, o.n_hcnc, 0);
    host_ms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
    // uploads on their own stream (they overlap the previous launch's kernels; this slot's arenas and buffers were
    // last used by the launch before that one, whose results decide() has already waited for); batch_init writes
    // [common, mut_end) of the arenas, the overlays [0, common)
    HIPCHK(hipMemcpy2DAsync(arenas, gb.stride, patches, patch_bytes, patch_bytes, n, hipMemcpyHostToDevice, up));
    HIPCHK(hipMemcpyAsync(dargs, reinterpret_cast<uint8_t*>(sl.up.at(u_args)), sizeof(SolveArgs) * n, hipMemcpyHostToDevice, up));
    HIPCHK(hipMemcpyAsync(dfargs, reinterpret_cast<uint8_t*>(sl.up.at(u_fargs)), sizeof(FinalizeArgs) * n, hipMemcpyHostToDevice, up));
    HIPCHK(hipEventRecord(sl.uploaded, up));
    hipStream_t ks = gb.cs.k[launch_no & 1];  // (the slot's kernel stream)
    HIPCHK(launch_batch_init(bi, n, ks));
    HIPCHK(hipStreamWaitEvent(ks, sl.uploaded, 0));
    HIPCHK(hipEventRecord(sl.t0, ks));
    HIPCHK(launch_solve_batch(sargs[0], dargs, n, dyn, ks));
    HIPCHK(launch_finalize_batch(fargs[0], dfargs, n, ks));
    HIPCHK(hipEventRecord(sl.t1, ks));
    // downloads on their own stream once the kernels are done (the next launch's kernels need not wait for them)
    HIPCHK(hipStreamWaitEvent(dn, sl.t1, 0));
    auto down = [&](size_t roff, size_t off, size_t width) {
      return hipMemcpy2DAsync(reinterpret_cast<uint8_t*>(sl.down.at(roff)), width, arenas + off, gb.stride, width, n, hipMemcpyDeviceToHost, dn);
    };
    HIPCHK(down(r_stats, o.stats, sizeof(uint64_t) * KP_SOLVE_STATS));
    HIPCHK(down(r_place, o.place, sizeof(int32_t) * Pc));
    HIPCHK(down(r_nct, o.nct, sizeof(int32_t)));
    HIPCHK(down(r_nopt, o.nopt, sizeof(uint32_t)));
    HIPCHK(down(r_opts, o.opts, sizeof(uint32_t) * gb.opt_stride));
    HIPCHK(down(r_fin, o.ncr, sizeof(KReqs)));
    if (gb.res_mode) HIPCHK(down(r_held, o.held, sizeof(uint64_t)));
    HIPCHK(hipEventRecord(sl.done, dn));
    sl.n = n;
    sl.b0 = b0;
    // the previous launch's decisions while this one runs
    if (pending >= 0) {
      if (int32_t rc = decide(slots[pending])) return rc;
    }
    pending = launch_no & 1;
    ++*n_launches;
  }
  if (pending >= 0) {
    if (int32_t rc = decide(slots[pending])) return rc;
  }
  return KP_OK;
}

static int32_t GeneralSimLocked(kp_cluster_plan* plan, const uint32_t* offsets, const uint32_t* nodes,
                                uint32_t n_subsets, int32_t multi_node, SimArgs& a, kp_cancel* cancel) {
  kp_ctx* ctx = plan->ctx;
  const kp_cluster& cl = plan->general->cl;
  const int N = (int)cl.n_nodes;
  if (int32_t rc = CatalogsAlive(plan->general->alive)) return rc;
  if (offsets[0] != 0) return fail(KP_E_INVAL, "offsets[0] != 0");
  if (offsets[n_subsets] && !nodes) return fail(KP_E_INVAL, "null nodes");
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  vector<std::map<string, string>>& labels = plan->general_labels;  // the nodes' labels (NodeCandidatePrice), once
  if ((int)labels.size() != N) {
    labels.assign(N, {});
    for (int i = 0; i < N; i++)
      for (uint32_t j = 0; j < cl.nodes[i].node.n_labels; j++) {
        const kp_label& l = cl.nodes[i].node.labels[j];
        labels[i][Normalize(l.key ? l.key : "")] = l.value ? l.value : "";
      }
  }
  for (uint32_t s = 0; s < n_subsets; s++)
    if (offsets[s + 1] < offsets[s]) return fail(KP_E_INVAL, "offsets not monotone at %u", s);
  // the subsets' candidate lists, checked on up to 16 threads (each with its own membership marks); the error reported
  // is the first subset's, as the serial check would report it
  vector<vector<uint32_t>> cands(n_subsets);
  std::atomic<int64_t> bad_s{INT64_MAX};
  vector<vector<char>> inS(kMaxHostThreads);
  ParallelFor((int)n_subsets, [&](int s_lo, int s_hi, int t) {
    vector<char>& mark = inS[t];
    mark.assign(N, 0);
    for (int s = s_lo; s < s_hi; s++) {
      cands[s].assign(nodes + offsets[s], nodes + offsets[s + 1]);
      bool ok = true;
      size_t k = 0;
      for (; k < cands[s].size(); k++) {
        const uint32_t c = cands[s][k];
        if (c >= (uint32_t)N || cl.nodes[c].deleting || mark[c]) {
          ok = false;
          break;
        }
        mark[c] = 1;
      }
      for (size_t j = 0; j < k; j++) mark[cands[s][j]] = 0;
      if (!ok) {
        int64_t cur = bad_s.load();
        while (s < cur && !bad_s.compare_exchange_weak(cur, s)) {
        }
        return;
      }
    }
  });
  if (bad_s.load() != INT64_MAX) {  // the serial check's message for the first bad subset
    const uint32_t s = (uint32_t)bad_s.load();
    vector<char> mark(N, 0);
    for (uint32_t k = offsets[s]; k < offsets[s + 1]; k++) {
      const uint32_t c = nodes[k];
      if (c >= (uint32_t)N) return fail(KP_E_INVAL, "subset %u: node %u", s, c);
      if (cl.nodes[c].deleting) return fail(KP_E_INVAL, "subset %u: node %u is being deleted", s, c);
      if (mark[c]) return fail(KP_E_INVAL, "subset %u: node %u twice", s, c);
      mark[c] = 1;
    }
  }
  // the batched path: built once per plan (again after an offering refresh of its catalogues)
  if (plan->gb) {
    const SolveBase& B = *plan->gb->C->B;
    if (CatalogsAlive(B.alive) || plan->gb->base_version != B.version || SeqnumsOf(B.catalogs) != B.seqnums) {
      plan->gb.reset();
      plan->gb_tried = false;
    }
  }
  const bool batch_on = ctx->ov.general_batch == 0;
  if (batch_on && !plan->gb_tried) {
    plan->gb_tried = true;
    int32_t rc = GeneralBatchBuild(plan, plan->gb);
    if (rc == KP_E_NOMEM || rc == KP_E_DEVICE) (void)hipGetLastError(), rc = KP_E_UNSUPPORTED;  // (as at prepare)
    if (rc && rc != KP_E_UNSUPPORTED) return rc;
    if (rc) plan->gb.reset();
  }
  const double t_setup = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  vector<SimOut> outs(n_subsets);
  memset(outs.data(), 0, sizeof(SimOut) * outs.size());
  uint64_t counters[3] = {0, 0, 0}, n_launches = 0;
  memset(plan->general_phase, 0, sizeof plan->general_phase);
  double dev_ms = 0, host_ms[2] = {0, 0};  // the batch's host work: overlays + arguments, decisions
  vector<int> batched, single;
  vector<char> batchable(n_subsets, 0);
  ParallelFor((int)n_subsets, [&](int s_lo, int s_hi, int) {
    for (int s = s_lo; s < s_hi; s++) {
      bool ok = batch_on && plan->gb;
      if (ok && plan->gb->C->G) {  // an inverse anti-affinity group would vanish: the per-subset compile
        const Compiled& C = *plan->gb->C;
        std::map<int, int> inv;
        for (uint32_t c : cands[s])
          for (int32_t g : C.node_inv[plan->gb->node_input[c]])
            if (++inv[g] == C.tg_inv_total[g]) ok = false;
      }
      batchable[s] = ok ? 1 : 0;
    }
  });
  for (uint32_t s = 0; s < n_subsets; s++) (batchable[s] ? batched : single).push_back((int)s);
  const auto t1 = clk::now();
  if (!batched.empty()) {
    const int32_t rc = GeneralBatchRun(plan, *plan->gb, cands, batched, labels, multi_node, outs, counters, &dev_ms, host_ms,
                                       cancel, &n_launches);
    if (rc) return rc;
  }
  const double t_batch = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
  const auto t2 = clk::now();
  for (int s : single) {
    const int32_t rc = GeneralSimOne(plan, cands[s], labels, multi_node, outs[s], counters, &dev_ms, cancel);
    if (rc) return rc;
  }
  const double t_single = std::chrono::duration<double, std::milli>(clk::now() - t2).count();
  // results and counters in device buffers, as the batched kernel leaves them
  const size_t need = sizeof(SimOut) * std::max<uint32_t>(n_subsets, 1) + 256 + sizeof(uint64_t) * 8;
  if (need > plan->batch_bytes) {
    if (plan->batch.p) HIPCHK(hipFree(plan->batch.p));
    plan->batch.p = nullptr;
    HIPCHK(hipMalloc(&plan->batch.p, need));
    plan->batch_bytes = need;
  }
  a = SimArgs{};
  a.out = (SimOut*)plan->batch.p;
  a.stats = (uint64_t*)((uint8_t*)plan->batch.p + ((sizeof(SimOut) * std::max<uint32_t>(n_subsets, 1) + 255) & ~(size_t)255));
  uint64_t st[8] = {counters[0], counters[1], counters[2], (uint64_t)batched.size(), (uint64_t)single.size(), 0, n_launches,
                    0};
  if (n_subsets) HIPCHK(hipMemcpyAsync(a.out, outs.data(), sizeof(SimOut) * n_subsets, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipMemcpyAsync(a.stats, st, sizeof st, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  plan->general_ms = dev_ms;
  plan->general_batched = (uint32_t)batched.size();
  if (ctx->ov.host_timing)
    fprintf(stderr, "[kp general] %u sims (%zu batched, %zu single): setup %.2f batch %.2f (overlays %.2f decisions %.2f "
            "device %.2f) single %.2f ms\n", n_subsets, batched.size(), single.size(), t_setup, t_batch, host_ms[0],
            host_ms[1], dev_ms, t_single);
  return KP_OK;
}

static int32_t SimLaunchLocked(kp_cluster_plan* plan, const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                               int32_t multi_node, SimArgs& a_out, kp_cancel* cancel) {
  kp_ctx* ctx = plan->ctx;
  if (cancel && __atomic_load_n(cancel->flag, __ATOMIC_SEQ_CST))
    return fail(KP_E_CANCELED, "cancelled before the simulations");
  if (plan->general) return GeneralSimLocked(plan, offsets, nodes, n_subsets, multi_node, a_out, cancel);
  if (int32_t rc = CatalogsAlive(plan->cp->B->alive)) return rc;
  if (SeqnumsOf(plan->cp->B->catalogs) != plan->cp->B->seqnums)
    return fail(KP_E_INVAL, "stale plan: a catalogue's seqnum changed since it was prepared (kp_cluster_refresh)");
  if (offsets[0] != 0) return fail(KP_E_INVAL, "offsets[0] != 0");
  const uint32_t n_flat = offsets[n_subsets];
  if (n_flat && !nodes) return fail(KP_E_INVAL, "null nodes");
  int cap = 1;
  const bool any_deleting = plan->n_base > 0;
  for (uint32_t s = 0; s < n_subsets; s++) {
    if (offsets[s + 1] < offsets[s]) return fail(KP_E_INVAL, "offsets not monotone at %u", s);
    uint64_t np = (uint64_t)plan->n_base;  // every simulation also schedules the pending and deleting-node pods
    for (uint32_t j = offsets[s]; j < offsets[s + 1]; j++) {
      if (nodes[j] >= (uint32_t)plan->N) return fail(KP_E_INVAL, "subset %u: node %u", s, nodes[j]);
      if (any_deleting && plan->deleting[nodes[j]]) return fail(KP_E_INVAL, "subset %u: node %u is being deleted", s, nodes[j]);
      np += plan->node_npods[nodes[j]];
    }
    if (np > 65535) return fail(KP_E_UNSUPPORTED, "subset %u reschedules %llu pods (max 65535)", s, (unsigned long long)np);
    cap = std::max(cap, (int)np);
  }
  SimArgs& a = a_out;
  a = plan->a;
  int cap2 = 1;
  while (cap2 < std::max(cap, 2 * plan->T2)) cap2 <<= 1;
  a.cap = cap;
  a.cap2 = cap2;
  a.wave_lds = (int)(((size_t)16 * a.EW + (size_t)6 * cap2 + 15) & ~(size_t)15);
  a.multi_node = multi_node ? 1 : 0;
  a.cancel = nullptr;
  if (cancel) {
    void* dp = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dp, cancel->flag, 0));
    a.cancel = (const int32_t*)dp;
  }
  hipFuncAttributes fa;
  HIPCHK(hipFuncGetAttributes(&fa, sim_kernel_ptr()));
  const size_t lds_wg = fa.sharedSizeBytes + (size_t)SIM_WAVES * a.wave_lds;
  if (lds_wg > 160 * 1024) return fail(KP_E_UNSUPPORTED, "simulation LDS %zu B per workgroup (cluster or subsets too large)", lds_wg);
  const int wg_per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / lds_wg));
  int blocks = std::min<int>((int)((n_subsets + SIM_WAVES - 1) / SIM_WAVES), plan->n_cu * wg_per_cu);
  blocks = std::max(blocks, 1);
  const int slots = blocks * SIM_WAVES;
  a.n_slots = slots;
  a.n_subsets = (int32_t)n_subsets;
  // per-wave scratch
  const size_t sz_pod = sizeof(uint64_t) * (size_t)slots * cap;
  const size_t sz_start = sizeof(int32_t) * (size_t)slots * std::max(a.SL, 1);
  const size_t sz_ovl = sizeof(int64_t) * (size_t)slots * std::max(a.E, 1) * std::max(a.RU, 1);
  const size_t sz_nc = sizeof(SimNC) * (size_t)slots;
  const size_t sz_fail = sizeof(int32_t) * (size_t)slots * std::max(a.SL, 1);
  const size_t sz_ovlhp = a.hp_any ? sizeof(uint64_t) * (size_t)slots * std::max(a.E, 1) : 8;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t need = al(sz_pod) + al(sz_start) + al(sz_ovl) + al(sz_nc) + al(sz_fail) + al(sz_ovlhp) + al(sizeof(uint64_t) * 8);
  if (need > plan->scratch_bytes) {
    if (plan->scratch.p) HIPCHK(hipFree(plan->scratch.p));
    plan->scratch.p = nullptr;
    HIPCHK(hipMalloc(&plan->scratch.p, need));
    plan->scratch_bytes = need;
  }
  uint8_t* sb = (uint8_t*)plan->scratch.p;
  size_t o = 0;
  a.s_pod = (uint64_t*)(sb + o);
  o += al(sz_pod);
  a.s_start = (int32_t*)(sb + o);
  o += al(sz_start);
  a.s_ovl = (int64_t*)(sb + o);
  o += al(sz_ovl);
  a.s_nc = (SimNC*)(sb + o);
  o += al(sz_nc);
  a.s_ncfail = (int32_t*)(sb + o);
  o += al(sz_fail);
  a.s_ovlhp = (uint64_t*)(sb + o);
  o += al(sz_ovlhp);
  a.stats = (uint64_t*)(sb + o);
  // batch: subsets + results
  const size_t b_off = al(sizeof(uint32_t) * (n_subsets + 1)), b_nodes = al(sizeof(uint32_t) * std::max<uint32_t>(n_flat, 1));
  const size_t b_out = al(sizeof(SimOut) * n_subsets);
  if (b_off + b_nodes + b_out > plan->batch_bytes) {
    if (plan->batch.p) HIPCHK(hipFree(plan->batch.p));
    plan->batch.p = nullptr;
    HIPCHK(hipMalloc(&plan->batch.p, b_off + b_nodes + b_out));
    plan->batch_bytes = b_off + b_nodes + b_out;
  }
  uint8_t* bb = (uint8_t*)plan->batch.p;
  a.sub_off = (const uint32_t*)bb;
  a.sub_nodes = (const uint32_t*)(bb + b_off);
  a.out = (SimOut*)(bb + b_off + b_nodes);
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(bb, offsets, sizeof(uint32_t) * (n_subsets + 1), hipMemcpyHostToDevice, st));
  if (n_flat) HIPCHK(hipMemcpyAsync(bb + b_off, nodes, sizeof(uint32_t) * n_flat, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(a.s_ncfail, 0xFF, sz_fail, st));
  HIPCHK(hipMemsetAsync(a.stats, 0, sizeof(uint64_t) * 8, st));
  HIPCHK(hipEventRecord(ctx->ev0, st));
  HIPCHK(launch_sim(a, blocks, (size_t)SIM_WAVES * a.wave_lds, st));
  HIPCHK(hipEventRecord(ctx->ev1, st));
  return KP_OK;
}

int32_t kp_cluster_simulate(kp_cluster_plan* plan, const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                            int32_t multi_node, kp_sim_result* out, kp_solve_stats* stats) {
  return kp_cluster_simulate_cancellable(plan, nullptr, offsets, nodes, n_subsets, multi_node, out, stats);
}

int32_t kp_cluster_simulate_cancellable(kp_cluster_plan* plan, kp_cancel* cancel, const uint32_t* offsets,
                                        const uint32_t* nodes, uint32_t n_subsets, int32_t multi_node, kp_sim_result* out,
                                        kp_solve_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!plan || (n_subsets && (!offsets || !out))) return fail(KP_E_INVAL, "null argument");
  if (cancel && cancel->ctx.p != plan->ctx.p) return fail(KP_E_INVAL, "the cancel token belongs to another context");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (stats) memset(stats, 0, sizeof *stats);
  if (n_subsets == 0) return KP_OK;
  SimArgs a;
  int32_t rc = SimLaunchLocked(plan, offsets, nodes, n_subsets, multi_node, a, cancel);
  if (rc) return rc;
  hipStream_t st = ctx->stream;
  uint64_t kst[8];
  HIPCHK(hipMemcpyAsync(out, a.out, sizeof(SimOut) * n_subsets, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(kst, a.stats, sizeof kst, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (!plan->general && kst[5]) return fail(KP_E_CANCELED, "consolidation simulations cancelled (kp_cancel_set)");
  float ms = (float)plan->general_ms;
  if (!plan->general) HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  for (uint32_t s = 0; s < n_subsets; s++)
    if (out[s].n_pods == 0xFFFFFFFFu) return fail(KP_E_DEVICE, "subset %u overflowed the pod queue", s);
  if (stats) {
    stats->device_ms = ms;
    stats->solve_kernel_ms = ms;
    stats->attempts = kst[0];
    stats->bytes_algorithmic = kst[1];
    stats->pops = kst[2];
    stats->phase_cycles[0] = kst[3];
    if (plan->general) {  // general path: simulations batched / compiled per subset, batched launches
      stats->phase_cycles[1] = kst[4];
      stats->phase_cycles[2] = kst[6];
      for (int k = 0; k < 8; k++) stats->attempt_cycles[k] = plan->general_phase[k];  // (timing diagnostics)
    }
    stats->prepare_ms = plan->prepare_ms;
    stats->host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return KP_OK;
}

int32_t kp_simulate_batch(kp_ctx* ctx, const kp_cluster* cl, const uint32_t* offsets, const uint32_t* nodes,
                          uint32_t n_subsets, int32_t multi_node, kp_sim_result* out, kp_solve_stats* stats) {
  kp_cluster_plan* plan = nullptr;
  int32_t rc = kp_cluster_prepare(ctx, cl, &plan);
  if (rc) return rc;
  const double prep = plan->prepare_ms;
  rc = kp_cluster_simulate(plan, offsets, nodes, n_subsets, multi_node, out, stats);
  if (stats) stats->prepare_ms = prep;
  kp_cluster_plan_destroy(plan);
  return rc;
}

}  // extern "C"

// ==================================================================================================
// Multi-GPU consolidation: RCCL communicator + the sweep's argmin (kp_consolidate_argmin)
// ==================================================================================================
static_assert(sizeof(kp_choice) == sizeof(CommBest), "kp_choice mirrors CommBest (the all-gathered record)");


namespace {
int32_t nccl_fail(ncclResult_t r, const char* what) {
  return fail(KP_E_DEVICE, "%s: %s", what, ncclGetErrorString(r));
}
// (savings desc, global index asc) over the records holding a decision (index >= 0)
bool Better(const kp_choice& x, const kp_choice& best) {
  if (x.subset < 0) return false;
  if (best.subset < 0) return true;
  if (x.result.savings != best.result.savings) return x.result.savings > best.result.savings;
  return x.subset < best.subset;
}
}  // namespace

extern "C" {

int32_t kp_choice_reduce(const kp_choice* per_rank, uint32_t n, kp_choice* out) {
  if (!out || (!per_rank && n)) return fail(KP_E_INVAL, "null argument");
  kp_choice best;
  memset(&best, 0, sizeof best);
  best.subset = -1;
  uint64_t counts[3] = {0, 0, 0}, overflowed = 0;
  for (uint32_t i = 0; i < n; i++)
    if (per_rank[i].subset == KP_CHOICE_FAILED)
      return fail(KP_E_DEVICE, "rank %u failed its step of the sweep (error %lld)", i, (long long)per_rank[i].counts[0]);
  for (uint32_t i = 0; i < n; i++) {
    for (int k = 0; k < 3; k++) counts[k] += per_rank[i].counts[k];
    overflowed += per_rank[i].overflowed;
    if (Better(per_rank[i], best)) best = per_rank[i];
  }
  for (int k = 0; k < 3; k++) best.counts[k] = counts[k];
  best.overflowed = overflowed;
  if (best.subset < 0) memset(&best.result, 0, sizeof best.result);
  *out = best;
  return KP_OK;
}

int32_t kp_comm_unique_id(uint8_t* id) {
  if (!id) return fail(KP_E_INVAL, "null argument");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  static_assert(sizeof(u) == KP_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof u);
  return KP_OK;
}

int32_t kp_comm_init(kp_ctx* ctx, const uint8_t* id, int32_t n_ranks, int32_t rank, kp_comm** out) {
  if (!ctx || !id || !out) return fail(KP_E_INVAL, "null argument");
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(KP_E_INVAL, "rank %d of %d", rank, n_ranks);
  HIPCHK(hipSetDevice(ctx->device));
  auto c = std::make_unique<kp_comm>();
  c->ctx = ctx;
  c->n_ranks = n_ranks;
  c->rank = rank;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, u, rank);
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitRank");
  HIPCHK(c->buf.alloc(sizeof(CommBest) * (size_t)(n_ranks + 1)));
  CommReadSettings(c.get());
  *out = c.release();
  return KP_OK;
}

int32_t kp_comm_init_all(kp_ctx* const* ctxs, int32_t n, kp_comm** out) {
  if (!ctxs || !out || n < 1) return fail(KP_E_INVAL, "null argument");
  vector<int> devs(n);
  for (int i = 0; i < n; i++) {
    if (!ctxs[i]) return fail(KP_E_INVAL, "null context %d", i);
    devs[i] = ctxs[i]->device;
    for (int j = 0; j < i; j++)
      if (devs[j] == devs[i]) return fail(KP_E_INVAL, "contexts %d and %d share GPU %d (RCCL: one rank per GPU)", j, i, devs[i]);
  }
  vector<ncclComm_t> comms(n, nullptr);
  ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitAll");
  vector<std::unique_ptr<kp_comm>> cs(n);
  for (int i = 0; i < n; i++) {
    cs[i] = std::make_unique<kp_comm>();
    cs[i]->ctx = ctxs[i];
    cs[i]->comm = comms[i];
    cs[i]->n_ranks = n;
    cs[i]->rank = i;
    CommReadSettings(cs[i].get());
  }
  for (int i = 0; i < n; i++) {
    if (hipSetDevice(devs[i]) != hipSuccess || cs[i]->buf.alloc(sizeof(CommBest) * (size_t)(n + 1)) != hipSuccess) {
      for (int j = 0; j < n; j++) (void)ncclCommDestroy(comms[j]);
      return fail(KP_E_NOMEM, "communicator buffer on GPU %d", devs[i]);
    }
  }
  for (int i = 0; i < n; i++) out[i] = cs[i].release();
  return KP_OK;
}

int32_t kp_comm_init_host(kp_ctx* ctx, int32_t n_ranks, int32_t rank, kp_allgather_fn fn, void* user, kp_comm** out) {
  if (!ctx || !fn || !out) return fail(KP_E_INVAL, "null argument");
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(KP_E_INVAL, "rank %d of %d", rank, n_ranks);
  auto c = std::make_unique<kp_comm>();
  c->ctx = ctx;
  c->host_fn = fn;
  c->host_user = user;
  c->n_ranks = n_ranks;
  c->rank = rank;
  CommReadSettings(c.get());
  *out = c.release();
  return KP_OK;
}

int32_t kp_comm_rank(const kp_comm* c, int32_t* rank, int32_t* n_ranks) {
  if (!c) return fail(KP_E_INVAL, "null argument");
  if (rank) *rank = c->rank;
  if (n_ranks) *n_ranks = c->n_ranks;
  return KP_OK;
}

void kp_comm_destroy(kp_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->ctx->device);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int32_t kp_consolidate_argmin(kp_cluster_plan* plan, kp_comm* comm, const uint32_t* offsets, const uint32_t* nodes,
                              uint32_t n_subsets, uint64_t base_index, int32_t multi_node, kp_sim_result* out,
                              kp_choice* best, kp_solve_stats* stats) {
  return kp_consolidate_argmin_cancellable(plan, comm, nullptr, offsets, nodes, n_subsets, base_index, multi_node, out,
                                           best, stats);
}

int32_t kp_consolidate_argmin_cancellable(kp_cluster_plan* plan, kp_comm* comm, kp_cancel* cancel,
                                          const uint32_t* offsets, const uint32_t* nodes, uint32_t n_subsets,
                                          uint64_t base_index, int32_t multi_node, kp_sim_result* out, kp_choice* best,
                                          kp_solve_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!plan || !best || (n_subsets && !offsets)) return fail(KP_E_INVAL, "null argument");
  if (cancel && cancel->ctx.p != plan->ctx.p) return fail(KP_E_INVAL, "the cancel token belongs to another context");
  if (comm && comm->ctx->device != plan->ctx->device) return fail(KP_E_INVAL, "comm and plan are on different GPUs");
  kp_ctx* ctx = plan->ctx;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  if (stats) memset(stats, 0, sizeof *stats);
  hipStream_t st = ctx->stream;
  float ms = 0;
  uint64_t kst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  CommBest mine;  // this rank's record (host)
  memset(&mine, 0, sizeof mine);
  DevBuf rec, parts;
  // the local step: simulation + device argmax into one record; any failure becomes a KP_CHOICE_FAILED record so that
  // the collective below is still reached by every rank
  auto local = [&]() -> int32_t {
    HIPCHK(hipSetDevice(ctx->device));
    SimArgs a;
    memset(&a, 0, sizeof a);
    const int n_parts = (int)std::min<uint32_t>(std::max<uint32_t>((n_subsets + 4095) / 4096, 1), 1024);
    HIPCHK(parts.alloc(sizeof(ArgmaxPart) * n_parts));
    HIPCHK(rec.alloc(sizeof(CommBest)));
    if (n_subsets) {
      int32_t rc = SimLaunchLocked(plan, offsets, nodes, n_subsets, multi_node, a, cancel);
      if (rc) return rc;
      if (out) HIPCHK(hipMemcpyAsync(out, a.out, sizeof(SimOut) * n_subsets, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(kst, a.stats, sizeof kst, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(launch_argmax(n_subsets ? a.out : nullptr, (int)n_subsets, (ArgmaxPart*)parts.p, n_parts,
                         (int64_t)base_index, (CommBest*)rec.p, st));
    HIPCHK(hipMemcpyAsync(&mine, rec.p, sizeof mine, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (n_subsets && !plan->general && kst[5])
      return fail(KP_E_CANCELED, "consolidation sweep cancelled (kp_cancel_set)");
    if (n_subsets && plan->general) ms = (float)plan->general_ms;
    else if (n_subsets) HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    return KP_OK;
  };
  const int32_t lrc = local();
  if (lrc) {
    memset(&mine, 0, sizeof mine);
    mine.index = KP_CHOICE_FAILED;
    mine.counts[0] = (uint64_t)(int64_t)lrc;
  }
  const int nr = comm ? comm->n_ranks : 1;
  vector<CommBest> recs(nr);
  if (comm && nr > 1) {  // one collective: every rank's 88-byte record to every rank (RCCL over xGMI)
    const string err = g_err;
    int32_t rc = CommExchange(comm, &mine, recs.data(), sizeof mine);
    if (rc) return rc;
    g_err = err;
  } else {
    recs[0] = mine;
  }
  if (lrc) return lrc;
  for (int i = 0; i < nr; i++)
    if (recs[i].index != KP_CHOICE_FAILED && recs[i].counts[3])
      return fail(KP_E_DEVICE, "rank %d: %llu subsets overflowed the pod queue", i, (unsigned long long)recs[i].counts[3]);
  vector<kp_choice> ch(nr);
  memcpy(ch.data(), recs.data(), sizeof(kp_choice) * nr);
  int32_t rc = kp_choice_reduce(ch.data(), (uint32_t)nr, best);
  if (rc) return rc;
  if (stats) {
    stats->device_ms = ms;
    stats->solve_kernel_ms = ms;
    stats->attempts = kst[0];
    stats->bytes_algorithmic = kst[1];
    stats->pops = kst[2];
    stats->phase_cycles[0] = kst[3];
    if (plan->general) {  // general path: simulations batched / compiled per subset, batched launches
      stats->phase_cycles[1] = kst[4];
      stats->phase_cycles[2] = kst[6];
      for (int k = 0; k < 8; k++) stats->attempt_cycles[k] = plan->general_phase[k];  // (timing diagnostics)
    }
    stats->prepare_ms = plan->prepare_ms;
    stats->host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return KP_OK;
}

}  // extern "C"
