// kp_sim.hip — batched consolidation simulations (included by kp_kernels.hip; shares its wave helpers).
//
// Upstream disruption computeConsolidation(S) runs SimulateScheduling = Solve(pods of S, existing nodes =
// every node not in S) and turns the Results into delete / replace / no-op (SURVEY §3 CS3, §8a a19;
// R:website/content/en/preview/concepts/disruption.md:89-128). Thousands of subsets S probe the SAME
// cluster snapshot, so the snapshot is resident and each simulation is an overlay on it:
//
//  sim_usable_kernel  per shape-level sl: the existing nodes whose ExistingNode.CanAdd succeeds on the
//                     snapshot (taints, Requirements.Compatible without the well-known allowance, Fits).
//                     Node labels are single-valued In requirements, so Compatible is one dictionary-bit
//                     test per pod key (lane = node, ballot -> 64-node word).
//  sim_prep_kernel    per shape-level: the addToNewNodeClaim outcome (first NodeClaimTemplate whose Add
//                     succeeds, and the NodeClaim it creates), before the NodePool limits; sim_kernel applies
//                     filterByRemainingResources on the replacement against the pools' remaining budget.
//  sim_kernel         one WAVE per simulation, persistent over the batch. Per simulation: exclusion bitmap
//                     of S and a "touched" bitmap in LDS, the pods of S sorted into Queue order (bitonic
//                     sort of their global queue ranks in LDS), then the Solve loop:
//                       existing nodes  first set bit of usable[sl] & ~excluded at or after start[sl];
//                                       touched nodes re-check Fits against their overlay requests.
//                                       Nodes only lose capacity, so every position before the last
//                                       winner stays a failure for sl: start[sl] is monotone.
//                       in-flight       the single NodeClaim: merge_compatible + filter_types (exact, as
//                                       in solve_kernel), failure memo per (sl, NodeClaim version)
//                       new NodeClaim   the precomputed template outcome; a second NodeClaim makes the
//                                       result a no-op, so the simulation stops there.
//                     then the decision: TruncateInstanceTypes (cheapest compatible offering, name; LDS
//                     bitonic sort) + minValues, filterByPrice on WorstLaunchPrice, filterOutSameType.
//
// The host routes the clusters these kernels do not model to the general path (each subset a whole device Solve,
// batched one workgroup per subset on the cluster's superset Solve: kp_host.cpp GeneralBatch): topology spread and pod (anti-)affinity, a pod NotIn/DoesNotExist requirement on a
// key some node lacks (ExistingNode requirements could then grow a key, and CanAdd would no longer be a function of
// the snapshot), and catalogues holding capacity reservations (strict reservation accounting).

__device__ __forceinline__ void sim_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ double wave_min_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const double w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ double lane_bcast_f64(double v, int src) {
  return __longlong_as_double((long long)lane_bcast((uint64_t)__double_as_longlong(v), src));
}

// ReqView of a stored requirement set (final NodeClaim requirements, pod requirements)
__device__ __forceinline__ ReqView stored_view(const DevDict& D, const KReqs* R, uint64_t v) {
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
  return rv;
}

// stage one shape-level (requirements, requests, PVP slots) into this wave's LDS
__device__ __forceinline__ void stage_shape(const SimArgs& a, int sl, int shape, KReqs* sB, int64_t* spreq,
                                            int32_t* spslot) {
  const int lane = LANE;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(a.shape_reqs + (size_t)sl * sizeof(KReqs));
  uint64_t* dst = reinterpret_cast<uint64_t*>(sB);
  constexpr int NQ = (int)(sizeof(KReqs) / 8);
  for (int i = lane; i < NQ; i += 64) dst[i] = src[i];
  if (lane < KP_NRES) spreq[lane] = a.shape_requests[(size_t)shape * KP_NRES + lane];
  spslot[lane] = a.pvp_slot[(size_t)sl * KP_MAX_KEYS + lane];
}

// wave-wide bitonic sort of n2 (power of two) u32 keys in LDS, ascending
__device__ void wave_bitonic_u32(uint32_t* k, int n2) {
  const int lane = LANE;
  for (int sz = 2; sz <= n2; sz <<= 1)
    for (int j = sz >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < n2; i += 64) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint32_t x = k[i], y = k[ixj];
          if ((x > y) == ((i & sz) == 0)) {
            k[i] = y;
            k[ixj] = x;
          }
        }
      }
      wave_sync();
    }
}
// same for (u64 key, u32 tie) pairs
__device__ void wave_bitonic_kv(uint64_t* k, uint32_t* v, int n2) {
  const int lane = LANE;
  for (int sz = 2; sz <= n2; sz <<= 1)
    for (int j = sz >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < n2; i += 64) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t ki = k[i], kj = k[ixj];
          const uint32_t vi = v[i], vj = v[ixj];
          const bool gt = ki > kj || (ki == kj && vi > vj);
          if (gt == ((i & sz) == 0)) {
            k[i] = kj;
            k[ixj] = ki;
            v[i] = vj;
            v[ixj] = vi;
          }
        }
      }
      wave_sync();
    }
}

// ------------------------------------------------------------------------------------------------
// usable[sl][w]: ExistingNode.CanAdd on the snapshot for the 64 nodes of word w
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(SIM_WAVES * 64) void sim_usable_kernel(SimArgs a) {
  __shared__ DevDict D;
  __shared__ uint64_t s_allow[SIM_WAVES][KP_MAX_WORDS];
  block_copy(D, a.dict);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = LANE;
  const long items = (long)a.SL * a.EW;
  for (long it = (long)blockIdx.x * SIM_WAVES + wave; it < items; it += (long)gridDim.x * SIM_WAVES) {
    const int sl = (int)(it / a.EW), w = (int)(it % a.EW);
    const int shape = a.sl_shape[sl];
    const KReqs* B = reinterpret_cast<const KReqs*>(a.shape_reqs + (size_t)sl * sizeof(KReqs));
    const uint64_t v = lane < D.W ? B->vals[lane] : 0;
    const ReqView rv = stored_view(D, B, v);
    s_allow[wave][lane] = allowed_word(D, rv, v, vint_global(a.vint));
    wave_sync();
    const uint64_t negB = a.shape_negop[sl];
    const uint64_t tol = a.shape_tolerates[sl];
    const int e = w * 64 + lane;
    bool ok = e < a.E;
    if (ok) ok = (tol >> a.ex_taintset[e]) & 1;
    if (ok && a.hp_any) ok = !(a.ex_hp[e] & a.shape_hp_conf[shape]);  // HostPortUsage.Conflicts
    for (int r = 0; r < KP_NRES && ok; r++) {  // Fits(Merge(requests, pod), available)
      const int64_t av = a.ex_available[(size_t)e * KP_NRES + r];
      ok = av >= 0 && a.ex_requests[(size_t)e * KP_NRES + r] + a.shape_requests[(size_t)shape * KP_NRES + r] <= av;
    }
    uint64_t keys = B->present;
    while (ok && keys) {  // Requirements.Compatible(node labels, pod) without the well-known allowance
      const int k = __builtin_ctzll(keys);
      keys &= keys - 1;
      const uint16_t code = a.ex_code[(size_t)k * a.E + e];
      if (code == 0xFFFF) ok = (negB >> k) & 1;  // undefined on the node: only NotIn / DoesNotExist
      else ok = (s_allow[wave][code >> 6] >> (code & 63)) & 1;  // In{label} ∩ pod requirement non-empty
    }
    const uint64_t bal = __ballot(ok);
    if (lane == 0) a.usable[(size_t)sl * a.EW + w] = bal;
    wave_sync();
  }
}

// ------------------------------------------------------------------------------------------------
// tres[sl]: addToNewNodeClaim for a pod of shape-level sl (templates in weight order, first success)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void copy_u64(uint64_t* dst, const uint64_t* src, int n) {
  for (int i = LANE; i < n; i += 64) dst[i] = src[i];
}

__global__ __launch_bounds__(SIM_WAVES * 64) void sim_prep_kernel(SimArgs a) {
  __shared__ DevDict D;
  __shared__ WaveSlots slots[SIM_WAVES];
  __shared__ KReqs s_B[SIM_WAVES];
  __shared__ int64_t s_preq[SIM_WAVES][KP_NRES];
  __shared__ int32_t s_pslot[SIM_WAVES][KP_MAX_KEYS];
  __shared__ uint32_t s_scratch[SIM_WAVES][2 * KP_MAX_WORDS];
  __shared__ int32_t s_fitj[SIM_WAVES][KP_NRES];
  __shared__ RowPtr s_rl[SIM_WAVES][RL_CAP];
  __shared__ CatHdr s_hdr[8];
  __shared__ CatHdr s_hdrw[SIM_WAVES];
  block_copy(D, a.dict);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = LANE;
  for (int c = wave; c < min(a.n_catalogs, 8); c += SIM_WAVES) hdr_fill_wave((CatHdr LDS*)&s_hdr[c], &a.cats[c], D.C);
  __syncthreads();
  auto hdr = [&](int c) -> const CatHdr LDS* {
    if (c < 8) return (const CatHdr LDS*)&s_hdr[c];
    hdr_fill_wave((CatHdr LDS*)&s_hdrw[wave], &a.cats[c], D.C);
    wave_sync();
    return (const CatHdr LDS*)&s_hdrw[wave];
  };
  uint64_t bytes = 0;
  for (int sl = blockIdx.x * SIM_WAVES + wave; sl < a.SL; sl += gridDim.x * SIM_WAVES) {
    const int shape = a.sl_shape[sl];
    stage_shape(a, sl, shape, &s_B[wave], s_preq[wave], s_pslot[wave]);
    wave_sync();
    SimNC* out = &a.tres[sl];
    const uint64_t negB = a.shape_negop[sl];
    const uint64_t tol = a.shape_tolerates[sl];
    int won = -1;
    for (int t = 0; t < a.n_tmpl && won < 0; t++) {
      if (!((tol >> a.tmpl_taintset[t]) & 1)) continue;
      const int cat = a.tmpl_catalog[t];
      uint64_t X = lane < D.TW ? a.tmpl_X[(size_t)t * D.TW + lane] : 0;
      const uint32_t lim = a.tmpl_limit_present[t];
      if (lim) {  // filterByRemainingResources: every limited resource's capacity within the NodePool's remaining
        const int64_t* rem = a.tmpl_remaining + (size_t)t * KP_NRES;
        const int64_t* capv = a.cats[cat].cap;
        uint64_t m = X, keep = 0;
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          const int ty = lane * 64 + b;
          bool viable = true;
          for (int r = 0; r < KP_NRES; r++)
            if (((lim >> r) & 1) && capv[(size_t)r * D.T + ty] > rem[r]) viable = false;
          if (viable) keep |= 1ull << b;
        }
        X = keep;
      }
      if (!__ballot(X != 0)) continue;
      uint64_t m_v = 0;
      ReqView rv;
      bool ok = merge_compatible(D, reinterpret_cast<const KReqs*>(a.tmpl_reqs + (size_t)t * sizeof(KReqs)), &s_B[wave],
                                 negB, true, m_v, rv, &slots[wave], vint_global(a.vint));
      if (ok) {
        const uint64_t* pvp = a.shape_pvp + (size_t)a.pvp_base[sl * a.n_catalogs + cat] * D.TW;
        const int64_t q_lane = lane < KP_NRES ? a.tmpl_daemon[(size_t)t * KP_NRES + lane] + s_preq[wave][lane] : 0;
        X = filter_types(D, hdr(cat), rv, m_v, X, s_B[wave].present, pvp, s_pslot[wave], q_lane, 0, nullptr,
                         a.req_res_mask, vint_global(a.vint), s_scratch[wave], (RowPtr LDS*)s_rl[wave], &bytes, s_fitj[wave]);
        ok = __ballot(X != 0) != 0;
      }
      if (ok) {
        store_merged(&out->reqs, rv, m_v, D.W, D.KB);
        if (lane < KP_MAX_TYPE_WORDS) out->X[lane] = lane < D.TW ? X : 0;
        if (lane < KP_NRES) {
          out->requests[lane] = a.tmpl_daemon[(size_t)t * KP_NRES + lane] + s_preq[wave][lane];
          out->fitj[lane] = s_fitj[wave][lane];
          out->maxalloc[lane] = INT64_MAX;
        }
        wave_sync();
        store_maxalloc(a.cats[cat].alloc, lane < D.TW ? X : 0, D.T, a.req_res_mask, out->maxalloc);
        if (lane == 0) {
          out->tmpl = t;
          out->taintset = a.tmpl_taintset[t];
          out->ver = 0;
          out->hp = a.hp_any ? a.shape_hp_add[shape] : 0;
        }
        won = t;
      }
      wave_sync();
    }
    if (won < 0 && lane == 0) out->tmpl = -1;
    wave_sync();
  }
}

// ------------------------------------------------------------------------------------------------
// sim_kernel: one wave per simulation
// ------------------------------------------------------------------------------------------------
#ifndef SIM_WPE
#define SIM_WPE 0  // waves per SIMD the register allocation targets (0: the compiler's choice; tools/kp_diag.h)
#endif
#if SIM_WPE
#define SIM_OCCUPANCY __attribute__((amdgpu_waves_per_eu(SIM_WPE, SIM_WPE)))
#else
#define SIM_OCCUPANCY
#endif
template <int NW>
__global__ __launch_bounds__(NW * 64) SIM_OCCUPANCY void sim_kernel(SimArgs a) {
  __shared__ DevDict D;
  __shared__ WaveSlots slots[NW];
  __shared__ KReqs s_B[NW];
  __shared__ int64_t s_preq[NW][KP_NRES];
  __shared__ int32_t s_pslot[NW][KP_MAX_KEYS];
  __shared__ uint32_t s_scratch[NW][2 * KP_MAX_WORDS];
  __shared__ uint64_t s_mask[NW][KP_MAX_TYPE_WORDS];
  __shared__ int32_t s_fitj[NW][KP_NRES];
  __shared__ RowPtr s_rl[NW][RL_CAP];
  __shared__ CatHdr s_hdr[8];
  __shared__ CatHdr s_hdrw[NW];
  extern __shared__ uint64_t s_dyn64[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = LANE;
  block_copy(D, a.dict);
  __syncthreads();
  for (int c = wave; c < min(a.n_catalogs, 8); c += NW) hdr_fill_wave((CatHdr LDS*)&s_hdr[c], &a.cats[c], D.C);
  __syncthreads();
  auto hdr = [&](int c) -> const CatHdr LDS* {
    if (c < 8) return (const CatHdr LDS*)&s_hdr[c];
    hdr_fill_wave((CatHdr LDS*)&s_hdrw[wave], &a.cats[c], D.C);
    wave_sync();
    return (const CatHdr LDS*)&s_hdrw[wave];
  };
  const int EW = a.EW, SL = a.SL, cap = a.cap;
  uint8_t* wbase = reinterpret_cast<uint8_t*>(s_dyn64) + (size_t)wave * a.wave_lds;
  uint64_t* excl = reinterpret_cast<uint64_t*>(wbase);
  uint64_t* dirty = excl + EW;
  uint32_t* keys = reinterpret_cast<uint32_t*>(dirty + EW);
  uint16_t* ring = reinterpret_cast<uint16_t*>(keys + a.cap2);
  uint64_t* fkey = dirty + EW;                                   // option sort (after the pod loop)
  uint32_t* fidx = reinterpret_cast<uint32_t*>(fkey + a.cap2 / 2);
  const int slot = blockIdx.x * NW + wave;
  uint64_t* spod = a.s_pod + (size_t)slot * cap;
  int32_t* sstart = a.s_start + (size_t)slot * SL;
  int64_t* ovl = a.s_ovl + (size_t)slot * a.E * a.RU;
  uint64_t* ovlhp = a.hp_any ? a.s_ovlhp + (size_t)slot * a.E : nullptr;
  SimNC* nc = a.s_nc + slot;
  int32_t* ncfail = a.s_ncfail + (size_t)slot * SL;
  KReqs* sB = &s_B[wave];
  int64_t* spreq = s_preq[wave];
  uint64_t attempts = 0, bytes = 0, pops = 0, words = 0;
  int32_t vcount = 0;
  const uint32_t rmask = a.req_res_mask;

  bool cancelled = false;
  for (int sim = slot, it = 0; sim < a.n_subsets; sim += a.n_slots, it++) {
    // kp_cancel (consolidation timeouts): the flag every 8 subsets of this wave; a set flag ends the wave's share
    if ((it & 7) == 0 && cancel_set(a.cancel)) {
      cancelled = true;
      break;
    }
    const uint32_t s0 = a.sub_off[sim];
    const int ns = (int)(a.sub_off[sim + 1] - s0);
    for (int w = lane; w < EW; w += 64) {
      excl[w] = a.base_excl[w];  // deleting nodes are never destinations
      dirty[w] = 0;
    }
    for (int i = lane; i < a.n_base; i += 64) keys[i] = a.base_keys[i];  // pending + deleting-node pods
    wave_sync();
    // ---- exclusions, candidate prices, pods of S ------------------------------------------------
    for (int i = lane; i < ns; i += 64) {
      const int pos = a.node_pos[a.sub_nodes[s0 + i]];
      atomicOr((unsigned long long*)&excl[pos >> 6], 1ull << (pos & 63));
    }
    int n = a.n_base;
    bool overflow = false;
    for (int i0 = 0; i0 < ns; i0 += 64) {
      const int i = i0 + lane;
      uint32_t off = 0;
      int cnt = 0;
      if (i < ns) {
        const uint32_t c = a.sub_nodes[s0 + i];
        off = a.node_pod_off[c];
        cnt = (int)(a.node_pod_off[c + 1] - off);
      }
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
      }
      const int total = __shfl(incl, 63, 64);
      if (n + total > cap) {
        overflow = true;
        break;
      }
      const int at = n + incl - cnt;
      for (int j = 0; j < cnt; j++) keys[at + j] = a.pod_rank[a.node_pods[off + j]];
      n += total;
    }
    double candPrice = 0;
    int flags_and = 3;
    if (lane == 0) {  // getCandidatePrices: summed in candidate order (float addition order matters)
      for (int i = 0; i < ns; i++) {
        const uint32_t c = a.sub_nodes[s0 + i];
        candPrice += a.node_price[c];
        flags_and &= a.node_flags[c];
      }
    }
    candPrice = lane_bcast_f64(candPrice, 0);
    flags_and = __builtin_amdgcn_readlane(flags_and, 0);
    const bool priced = flags_and & 1, allSpot = (flags_and >> 1) & 1;
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = n + lane; i < n2; i += 64) keys[i] = 0xFFFFFFFFu;
    wave_sync();
    wave_bitonic_u32(keys, n2);  // Queue order byCPUAndMemoryDescending over the pods of S
    for (int i = lane; i < n; i += 64) {
      ring[i] = (uint16_t)i;
      spod[i] = 0;
    }
    for (int q = lane; q < SL; q += 64) sstart[q] = 0;
    sim_sync();

    // ---- the Solve loop -------------------------------------------------------------------------
    // need: pods that must schedule (all but the pending ones: AllNonPendingPodsScheduled)
    int need = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      const bool req = i < n && a.pod_kind[a.rank_pod[keys[i]]] != 2;
      need += __builtin_popcountll(__ballot(req));
    }
    int head = 0, len = overflow ? 0 : n, n_nc = 0, placed_cnt = 0;
    uint32_t epoch = 1;
    bool abort = overflow;
    while (len > 0) {
      const int i = ring[head];
      const uint64_t ent = spod[i];
      if ((uint32_t)(ent >> 40) == epoch && (int)(uint32_t)ent == len) break;  // Pop: no progress
      head = head + 1 == n ? 0 : head + 1;
      len--;
      pops++;
      const int lvl = (int)((ent >> 32) & 0xFF);
      const int gid = (int)a.rank_pod[keys[i]];
      const int kind = a.pod_kind[gid];
      const int shape = a.pod_shape[gid];
      const int sl = a.shape_level_base[shape] + lvl;
      stage_shape(a, sl, shape, sB, spreq, s_pslot[wave]);
      sim_sync();
      const uint64_t hpc = a.hp_any ? a.shape_hp_conf[shape] : 0, hpa = a.hp_any ? a.shape_hp_add[shape] : 0;
      int placed = -1;  // 0: the NodeClaim; <= -2: existing position -2-placed
      // addToExistingNode
      int st = sstart[sl];
      for (int w0 = st >> 6; w0 < EW; w0 += 64) {
        const int w = w0 + lane;
        uint64_t c = 0, d = 0;
        if (w < EW) {
          c = a.usable[(size_t)sl * EW + w] & ~excl[w];
          if (w == (st >> 6)) c &= ~0ull << (st & 63);
          d = c & dirty[w];
        }
        words++;
        const uint64_t cl = c & ~d;
        int found = -1;
        uint64_t dd = d & (cl ? (cl & (0 - cl)) - 1 : ~0ull);  // touched nodes before the first untouched one
        while (dd) {
          const int b = __builtin_ctzll(dd);
          dd &= dd - 1;
          const int e = w * 64 + b;
          bool fits = true;
          for (int u = 0; u < a.RU; u++) {
            const int r = a.ru_res[u];
            fits = fits && ovl[(size_t)e * a.RU + u] + spreq[r] <= a.ex_available[(size_t)e * KP_NRES + r];
          }
          if (hpc) fits = fits && !(ovlhp[e] & hpc);  // ports the simulation's pods took on the node
          if (fits) {
            found = b;
            break;
          }
        }
        if (found < 0 && cl) found = __builtin_ctzll(cl);
        const uint64_t bal = __ballot(found >= 0);
        if (bal) {
          const int L = __builtin_ctzll(bal);
          const int fb = __builtin_amdgcn_readlane(found, L);
          const int e = (w0 + L) * 64 + fb;
          placed = -2 - e;
          st = e;
          break;
        }
        st = (w0 + 64) * 64;
      }
      bytes += 8ull * 64;
      if (lane == 0) sstart[sl] = st;
      if (placed <= -2) {
        const int e = -2 - placed;
        if (!a.ex_init[e] && kind == 0) {
          abort = true;  // SimulateScheduling: a candidate pod relied on an uninitialized node
        } else {
          const bool first = !((dirty[e >> 6] >> (e & 63)) & 1);
          if (lane < a.RU) {
            const int r = a.ru_res[lane];
            const int64_t prev = first ? a.ex_requests[(size_t)e * KP_NRES + r] : ovl[(size_t)e * a.RU + lane];
            ovl[(size_t)e * a.RU + lane] = prev + spreq[r];
          }
          if (ovlhp && lane == 0) ovlhp[e] = (first ? a.ex_hp[e] : ovlhp[e]) | hpa;
          wave_sync();
          if (lane == 0) dirty[e >> 6] |= 1ull << (e & 63);
        }
        sim_sync();
      }
      // addToInflightNode (at most one NodeClaim exists)
      if (placed == -1 && n_nc == 1) {
        const uint64_t tol = a.shape_tolerates[sl];
        bool cand = ((tol >> nc->taintset) & 1) && ncfail[sl] != nc->ver && !(nc->hp & hpc);
        if (cand)
          for (int r = 0; r < KP_NRES; r++)
            if (((rmask >> r) & 1) && nc->requests[r] + spreq[r] > nc->maxalloc[r]) cand = false;
        if (cand) {
          attempts++;
          const int cat = a.tmpl_catalog[nc->tmpl];
          uint64_t m_v = 0, X = 0;
          ReqView rv;
          bool ok = merge_compatible(D, &nc->reqs, sB, a.shape_negop[sl], true, m_v, rv, &slots[wave],
                                     vint_global(a.vint));
          bytes += sizeof(KReqs);
          if (ok) {
            X = lane < D.TW ? nc->X[lane] : 0;
            const uint64_t* pvp = a.shape_pvp + (size_t)a.pvp_base[sl * a.n_catalogs + cat] * D.TW;
            const int64_t q_lane = lane < KP_NRES ? nc->requests[lane] + spreq[lane] : 0;
            const int32_t j0_lane = lane < KP_NRES ? nc->fitj[lane] : 0;
            X = filter_types(D, hdr(cat), rv, m_v, X, sB->present, pvp, s_pslot[wave], q_lane, j0_lane, nullptr,
                             rmask, vint_global(a.vint), s_scratch[wave], (RowPtr LDS*)s_rl[wave],
                             &bytes, s_fitj[wave]);
            ok = __ballot(X != 0) != 0;
          }
          if (ok) {
            store_merged(&nc->reqs, rv, m_v, D.W, D.KB);
            if (lane < D.TW) nc->X[lane] = X;
            if (lane < KP_NRES) {
              nc->requests[lane] += spreq[lane];
              nc->fitj[lane] = s_fitj[wave][lane];
            }
            if (lane == 0) nc->ver = ++vcount;
            if (lane == 0) nc->hp |= hpa;
            placed = 0;
          } else if (lane == 0) {
            ncfail[sl] = nc->ver;
          }
          sim_sync();
        }
      }
      // addToNewNodeClaim: precomputed outcome; a second NodeClaim makes the result a no-op
      if (placed == -1 && a.tres[sl].tmpl >= 0) {
        if (n_nc == 1) {
          abort = true;
        } else {
          copy_u64(reinterpret_cast<uint64_t*>(nc), reinterpret_cast<const uint64_t*>(&a.tres[sl]),
                   (int)(sizeof(SimNC) / 8));
          sim_sync();
          if (lane == 0) nc->ver = ++vcount;
          sim_sync();
          n_nc = 1;
          placed = 0;
        }
      }
      if (abort) break;
      if (placed != -1) {
        if (kind != 2) placed_cnt++;
      } else {  // Preferences.Relax + Queue.Push
        const bool relaxed = lvl + 1 < a.shape_nlevels[shape];
        int tail = head + len;
        if (tail >= n) tail -= n;
        len++;
        uint64_t ne;
        if (relaxed) {
          epoch++;  // lastLen = map{}
          ne = (uint64_t)(lvl + 1) << 32;
        } else {
          ne = ((uint64_t)epoch << 40) | ((uint64_t)lvl << 32) | (uint32_t)len;
        }
        if (lane == 0) {
          ring[tail] = (uint16_t)i;
          spod[i] = ne;
        }
        sim_sync();
      }
    }

    // ---- decision (computeConsolidation) ---------------------------------------------------------
    int decision = KP_DECISION_NOOP, nodepool = 0, n_options = 0;
    double repl = 0, savings = 0;
    const double candReported = priced ? candPrice : 0.0;
    if (!abort && placed_cnt == need) {
      if (n_nc == 0) {
        decision = KP_DECISION_DELETE;
        savings = candReported;
      } else if (priced) {
        const int cat = a.tmpl_catalog[nc->tmpl];
        const DevCatalog& Cg = a.cats[cat];
        const uint64_t v = lane < D.W ? nc->reqs.vals[lane] : 0;
        const ReqView rv = stored_view(D, &nc->reqs, v);
        const uint64_t negR = negop_mask(rv.present, rv.compl_, rv.nz);
        const uint64_t allowed = allowed_word(D, rv, v, vint_global(a.vint));
        const uint64_t cls = allowed_classes(D, Cg.cls, rv, allowed, negR);
        const bool ctp = (rv.present >> a.ct_key) & 1;
        bool ncSpot;
        if (a.spot_bit >= 0) ncSpot = !ctp || bit_of(allowed, a.spot_bit);
        else ncSpot = !ctp || ((rv.compl_ >> a.ct_key) & 1);
        // spot-to-spot (every candidate spot, the replacement may launch spot): only with the feature gate, on
        // the replacement narrowed to spot offerings, and a single candidate needs 15 cheaper options
        const bool s2s = allSpot && ncSpot;
        if (!s2s || a.spot_to_spot) {
          // TruncateInstanceTypes: OrderByPrice (cheapest compatible offering, then name) + cut
          const uint64_t Xl = lane < D.TW ? nc->X[lane] : 0;
          int cnt = 0;
          for (int ch = 0; ch < D.TW; ch++) {
            const uint64_t wd = lane_bcast(Xl, ch);
            const int t = ch * 64 + lane;
            const bool has = (wd >> lane) & 1;
            double p = __builtin_huge_val();
            if (has && Cg.price_sub) {  // min over the compatible class set in one gather
              p = Cg.price_sub[(size_t)cls * D.T + t];
            } else if (has) {
              uint64_t m = cls;
              while (m) {
                const int c = __builtin_ctzll(m);
                m &= m - 1;
                const double q = Cg.price[(size_t)t * D.C + c];
                p = q < p ? q : p;
              }
            }
            const uint64_t bal = __ballot(has);
            if (has) {
              const int pos = cnt + __builtin_popcountll(bal & ((1ull << lane) - 1));
              fkey[pos] = (uint64_t)__double_as_longlong(p);
              fidx[pos] = (Cg.name_rank[t] << 12) | (uint32_t)t;
            }
            cnt += __builtin_popcountll(bal);
          }
          int m2 = 1;
          while (m2 < cnt) m2 <<= 1;
          for (int q = cnt + lane; q < m2; q += 64) {
            fkey[q] = ~0ull;
            fidx[q] = ~0u;
          }
          wave_sync();
          wave_bitonic_kv(fkey, fidx, m2);
          const int lim = a.max_types ? min(cnt, a.max_types) : cnt;
          uint64_t* msk = s_mask[wave];
          const uint64_t hmin = rv.hmin & rv.present;
          bool ok = true;
          if (hmin) {  // minValues must survive the truncation, else the pods fail (no-op)
            msk[lane] = 0;
            wave_sync();
            for (int q = lane; q < lim; q += 64) {
              const uint32_t t = fidx[q] & 4095u;
              atomicOr((unsigned long long*)&msk[t >> 6], 1ull << (t & 63));
            }
            wave_sync();
            ok = minvalues_ok(D, Cg.code, Cg.TM, hmin, rv.minv, lane < D.TW ? msk[lane] : 0, s_scratch[wave]);
          }
          // filterByPrice: Offerings.Available().WorstLaunchPrice(reqs) < candidate price
          double wlp[2] = {__DBL_MAX__, __DBL_MAX__};
          int tt[2] = {-1, -1};
          for (int h = 0; h < 2; h++) {
            const int q = h * 64 + lane;
            if (q >= lim) continue;
            const int t = (int)(fidx[q] & 4095u);
            tt[h] = t;
            for (int pass = 0; pass < (s2s ? 1 : 2); pass++) {  // capacity-type precedence: spot, on-demand
              const int ctb = pass == 0 ? a.spot_bit : a.od_bit;
              if (ctb < 0) continue;
              bool any = false;
              double mx = 0;
              uint64_t m = cls;
              while (m) {
                const int c = __builtin_ctzll(m);
                m &= m - 1;
                if (Cg.cls[c].ct_bit != ctb || !((Cg.offer_avail[(size_t)c * D.TW + (t >> 6)] >> (t & 63)) & 1)) continue;
                const double pr = Cg.price[(size_t)t * D.C + c];
                if (!any || pr > mx) mx = pr;
                any = true;
              }
              if (any) {
                wlp[h] = mx;
                break;
              }
            }
          }
          bool keep[2] = {tt[0] >= 0 && wlp[0] < candPrice, tt[1] >= 0 && wlp[1] < candPrice};
          for (int stage = 0; stage < 2 && ok; stage++) {
            if (stage == 1) {
              if (!a.multi_node) break;
              // filterOutSameType: the cheapest candidate of a kept option's type caps the price
              double mp = __DBL_MAX__;
              for (int h = 0; h < 2; h++) {
                if (!keep[h]) continue;
                const uint32_t nm = a.type_name[(size_t)cat * D.T + tt[h]];
                for (int i = 0; i < ns; i++) {
                  const uint32_t c = a.sub_nodes[s0 + i];
                  if ((a.node_flags[c] & 1) && a.node_name[c] == nm && a.node_price[c] < mp) mp = a.node_price[c];
                }
              }
              const double maxPrice = wave_min_f64(mp);
              keep[0] = keep[0] && wlp[0] < maxPrice;
              keep[1] = keep[1] && wlp[1] < maxPrice;
            }
            const int count = wave_sum((keep[0] ? 1 : 0) + (keep[1] ? 1 : 0));
            if (hmin) {
              msk[lane] = 0;
              wave_sync();
              for (int h = 0; h < 2; h++)
                if (keep[h]) atomicOr((unsigned long long*)&msk[tt[h] >> 6], 1ull << (tt[h] & 63));
              wave_sync();
              if (!minvalues_ok(D, Cg.code, Cg.TM, hmin, rv.minv, lane < D.TW ? msk[lane] : 0, s_scratch[wave])) ok = false;
            }
            if (count == 0) ok = false;
            n_options = count;
          }
          if (ok && s2s && ns == 1) {  // MinInstanceTypesForSpotToSpotConsolidation, then the launch keeps 15
            if (n_options < 15) {
              ok = false;
            } else {  // the first 15 (100 with minValues) kept options in price order
              const int L = hmin ? 100 : 15;
              const uint64_t lt = (1ull << lane) - 1;
              const uint64_t b0 = __ballot(keep[0]), b1 = __ballot(keep[1]);
              keep[0] = keep[0] && __popcll(b0 & lt) < L;
              keep[1] = keep[1] && __popcll(b0) + __popcll(b1 & lt) < L;
              n_options = min(n_options, L);
            }
          }
          if (ok) {
            double b = __DBL_MAX__;
            for (int h = 0; h < 2; h++)
              if (keep[h] && wlp[h] < b) b = wlp[h];
            const double best = wave_min_f64(b);
            decision = KP_DECISION_REPLACE;
            nodepool = a.tmpl_nodepool[nc->tmpl];
            repl = best;
            savings = candPrice - best;
          } else {
            n_options = 0;
          }
        }
      }
    }
    if (lane == 0) {
      SimOut o;
      o.decision = decision;
      o.nodepool = (uint32_t)nodepool;
      o.candidate_price = candReported;
      o.replacement_price = repl;
      o.savings = savings;
      o.n_options = (uint32_t)(decision == KP_DECISION_REPLACE ? n_options : 0);
      o.n_pods = overflow ? 0xFFFFFFFFu : (uint32_t)n;
      a.out[sim] = o;
    }
    sim_sync();
  }
  if (lane == 0) {
    atomicAdd((unsigned long long*)&a.stats[0], (unsigned long long)attempts);
    atomicAdd((unsigned long long*)&a.stats[1], (unsigned long long)bytes);
    atomicAdd((unsigned long long*)&a.stats[2], (unsigned long long)pops);
    atomicAdd((unsigned long long*)&a.stats[3], (unsigned long long)words);
    if (cancelled) atomicAdd((unsigned long long*)&a.stats[5], 1ull);
  }
}

hipError_t launch_sim_prep(const SimArgs& a, hipStream_t s) {
  const long items = (long)a.SL * a.EW;
  long blocks = (items + SIM_WAVES - 1) / SIM_WAVES;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  if (a.EW > 0) hipLaunchKernelGGL(sim_usable_kernel, dim3((unsigned)blocks), dim3(SIM_WAVES * 64), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int pb = (a.SL + SIM_WAVES - 1) / SIM_WAVES;
  if (pb > 0) hipLaunchKernelGGL(sim_prep_kernel, dim3(pb), dim3(SIM_WAVES * 64), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_sim(const SimArgs& a, int blocks, size_t dyn_lds, hipStream_t s) {
  hipLaunchKernelGGL(sim_kernel<SIM_WAVES>, dim3(blocks), dim3(SIM_WAVES * 64), dyn_lds, s, a);
  return hipGetLastError();
}
const void* sim_kernel_ptr() { return reinterpret_cast<const void*>(sim_kernel<SIM_WAVES>); }

// ------------------------------------------------------------------------------------------------
// Best decision of a simulated batch (kp_consolidate_argmin): max savings over non-no-op decisions, ties to the
// lowest subset index, plus the decision counts. Two stages: blocks reduce contiguous ranges, one block the partials.
// ------------------------------------------------------------------------------------------------
#define ARGMAX_THREADS 256
__device__ __forceinline__ bool better(double s, int64_t i, double bs, int64_t bi) {
  return i >= 0 && (bi < 0 || s > bs || (s == bs && i < bi));
}
__global__ __launch_bounds__(ARGMAX_THREADS) void argmax_kernel(const SimOut* out, int n, ArgmaxPart* part) {
  __shared__ double s_s[ARGMAX_THREADS];
  __shared__ int64_t s_i[ARGMAX_THREADS];
  __shared__ unsigned long long s_cnt[4];
  const int tid = threadIdx.x;
  if (tid < 4) s_cnt[tid] = 0;
  __syncthreads();
  const int per = (n + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * per, hi = min(n, lo + per);
  double bs = 0;
  int64_t bi = -1;
  unsigned long long c[4] = {0, 0, 0, 0};
  for (int i = lo + tid; i < hi; i += ARGMAX_THREADS) {
    const SimOut o = out[i];
    const int d = o.decision;
    c[d == KP_DECISION_DELETE ? 1 : (d == KP_DECISION_REPLACE ? 2 : 0)]++;
    if (o.n_pods == 0xFFFFFFFFu) c[3]++;  // overflowed the pod queue (an error on the host)
    if (d != KP_DECISION_NOOP && better(o.savings, i, bs, bi)) bs = o.savings, bi = i;
  }
  s_s[tid] = bs;
  s_i[tid] = bi;
  for (int k = 0; k < 4; k++) atomicAdd(&s_cnt[k], c[k]);
  __syncthreads();
  for (int w = ARGMAX_THREADS / 2; w > 0; w >>= 1) {
    if (tid < w && better(s_s[tid + w], s_i[tid + w], s_s[tid], s_i[tid])) {
      s_s[tid] = s_s[tid + w];
      s_i[tid] = s_i[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    part[blockIdx.x].savings = s_s[0];
    part[blockIdx.x].index = s_i[0];
    for (int k = 0; k < 4; k++) part[blockIdx.x].counts[k] = s_cnt[k];
  }
}
// one block: partials -> the record this rank contributes to the all-gather
__global__ __launch_bounds__(ARGMAX_THREADS) void argmax_final_kernel(const ArgmaxPart* part, int np, const SimOut* out,
                                                                     int64_t base, CommBest* dst) {
  __shared__ double s_s[ARGMAX_THREADS];
  __shared__ int64_t s_i[ARGMAX_THREADS];
  __shared__ unsigned long long s_cnt[4];
  const int tid = threadIdx.x;
  if (tid < 4) s_cnt[tid] = 0;
  __syncthreads();
  double bs = 0;
  int64_t bi = -1;
  unsigned long long c[4] = {0, 0, 0, 0};
  for (int i = tid; i < np; i += ARGMAX_THREADS) {
    if (better(part[i].savings, part[i].index, bs, bi)) bs = part[i].savings, bi = part[i].index;
    for (int k = 0; k < 4; k++) c[k] += part[i].counts[k];
  }
  s_s[tid] = bs;
  s_i[tid] = bi;
  for (int k = 0; k < 4; k++) atomicAdd(&s_cnt[k], c[k]);
  __syncthreads();
  for (int w = ARGMAX_THREADS / 2; w > 0; w >>= 1) {
    if (tid < w && better(s_s[tid + w], s_i[tid + w], s_s[tid], s_i[tid])) {
      s_s[tid] = s_s[tid + w];
      s_i[tid] = s_i[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    dst->index = s_i[0] >= 0 ? base + s_i[0] : -1;
    if (s_i[0] >= 0) dst->rec = out[s_i[0]];
    else memset(&dst->rec, 0, sizeof(SimOut));
    for (int k = 0; k < 4; k++) dst->counts[k] = s_cnt[k];
  }
}
hipError_t launch_argmax(const SimOut* out, int n, ArgmaxPart* part, int n_parts, int64_t base, CommBest* dst,
                         hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(argmax_kernel, dim3(n_parts), dim3(ARGMAX_THREADS), 0, s, out, n, part);
  else (void)hipMemsetAsync(part, 0xFF, sizeof(ArgmaxPart) * n_parts, s);  // index -1 everywhere (counts fixed below)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(argmax_final_kernel, dim3(1), dim3(ARGMAX_THREADS), 0, s, part, n > 0 ? n_parts : 0, out, base, dst);
  return hipGetLastError();
}
