// gg_dev.h — device-side building blocks shared by the NoC (gg_noc.hip) and
// coherent (gg_coherent.hip) paths: the QueueModelHistoryTree restatement,
// the time conversions and the closed-form EMesh routes.
#pragma once
#include "gg_internal.h"

namespace gg {

// ---------------------------------------------------------------------------
// Queue models (QueueModel::create, queue_model.cc:19-39).  One storage
// layout for all three: HQueue + max_size 16-byte HNode slots.
//   history_tree (queue_model_history_tree.cc:44-167 over interval_tree.cc):
//     the free intervals sorted by start in a circular list of max_size
//     slots (interval i at slot (head + i) mod max_size), so the pruning of
//     the oldest interval is head + 1 and the usual update — at the newest
//     interval, the packets of a port arriving in time order — touches one
//     slot.  The reference keeps
//     them in an AVL tree and finds the interval with searchTree
//     (interval_tree.cc:366-394); the free intervals are disjoint and, since
//     every processing time and min_processing_time is >= 1 (router queues 1,
//     router_model.cc:23-27; DRAM 13, dram_perf_model.cc:48,92), separated by
//     at least one busy cycle and at least min_processing_time long.  For such
//     a set searchTree returns the FIRST interval (lowest start) that either
//     contains [t, t+p] or starts after t with length >= p, whatever the tree
//     shape: a left subtree it skips (t + p >= node start) holds only
//     intervals that end at or before the node's start, so none contains
//     [t, t+p] and none starting after t is long enough.  search(0, 1) is
//     then nd[0] (the min-key node the pruning removes, :52-56).  The
//     outputs (delays, analytical count, utilization) are those of the AVL
//     (tests/test_queue_flat.py checks 600k random requests against the
//     oracle's AVL restatement; the reference fixtures run on the GPU).
//   history_list (queue_model_history_list.cc:40-134): nd[0..size) in list order;
//   basic (queue_model_basic.cc:34-61): the MovingAverage window
//     (moving_average.h, window + 1 slots) as raw u64 words over nd[].
// ---------------------------------------------------------------------------
struct HNode { uint64_t first, second; };
struct HQueue {
  uint32_t size; uint32_t max_size; uint32_t type, aux;   // GG_QM_*; list: no-interleaving flag; basic: basic_moving_avg
  uint64_t sig_sq, sig, n, newest;                  // QueueModelMG1: sums of p^2 and p (integers, see mg1_queue_delay)
  uint64_t analytical;                              // _total_requests_using_analytical_model
  uint64_t util, last_req, total_req;               // QueueModel utilization counters
  uint32_t front, back;                             // basic: ModuloNum window ends (modulo window + 1)
  double mean;                                      // basic: MovingArithmeticMean::_arithmetic_mean
  uint64_t qtime;                                   // basic: QueueModelBasic::_queue_time
  uint32_t head, pad;                               // history_tree: slot of interval 0 (circular list)
};
static_assert(sizeof(HQueue) % 16 == 0 && sizeof(HNode) == 16, "16-byte queue images");

// the model-specific parameter of a queue of type `type` (gg_config fields)
__host__ __device__ inline uint32_t hq_aux(uint32_t type, uint32_t basic_moving_avg, uint32_t list_no_interleaving)
{
  return type == GG_QM_BASIC ? basic_moving_avg : list_no_interleaving;
}
__host__ __device__ inline uint32_t hq_window(uint32_t aux) { return (aux & 0xFFFFu) ? (aux & 0xFFFFu) : 64u; }

// host-side validation of a queue model configuration
inline gg_status gg_check_queue_model(uint32_t type, uint32_t aux, uint32_t max_size)
{
  if (type > GG_QM_BASIC) return gg_fail(GG_ERR_INVALID, "unknown queue model type");
  if (max_size < 2) return gg_fail(GG_ERR_UNSUPPORTED, "max_list_size below 2");
  if (type == GG_QM_BASIC) {
    if ((aux >> 16) == GG_MAVG_GEOMETRIC_MEAN) return gg_fail(GG_ERR_UNSUPPORTED, "geometric_mean moving average");
    if ((aux >> 16) > GG_MAVG_GEOMETRIC_MEAN) return gg_fail(GG_ERR_INVALID, "unknown moving average type");
    if (hq_window(aux) + 1 > 2 * max_size)
      return gg_fail(GG_ERR_UNSUPPORTED, "moving_avg_window_size + 1 exceeds 2 * max_list_size queue words");
  }
  return GG_OK;
}

// QueueModel{HistoryTree,HistoryList,Basic} constructors on one queue's storage
__device__ inline void hq_init(HQueue* q, HNode* N, uint32_t max_size, uint32_t type, uint32_t aux)
{
  HQueue Q{};
  Q.max_size = max_size;
  Q.type = type;
  Q.aux = aux;
  if (type == GG_QM_BASIC) {
    uint64_t* w = reinterpret_cast<uint64_t*>(N);
    for (uint32_t j = 0; j <= hq_window(aux); ++j) w[j] = 0;   // _num_list.resize(window + 1)
  } else {
    N[0].first = 0; N[0].second = ~0ull;            // history_tree: allocateNode(PAIR(0, UINT64_MAX));
    Q.size = 1;                                     // history_list: push_back(make_pair(0, UINT64_MAX))
  }
  *q = Q;
}

// One wave's lane id and wave-level ordering of LDS accesses between lanes.
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ void wave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint64_t ballot64(bool b) { return __ballot(b); }

// QueueModelMG1::computeQueueDelay (queue_model_m_g_1.cc).  The reference
// accumulates _service_time_sum(2) in doubles; every term is an integer
// processing time, so while the sums stay below 2^53 the double sums are the
// exact integers kept here (mg1_update flags GG_DERR_RANGE beyond).
__device__ __forceinline__ uint64_t mg1_queue_delay(uint64_t n, uint64_t newest, uint64_t ssq, uint64_t ss)
{
  if (n == 0) return 0;
  const double sig_sq = (double)ssq, sig = (double)ss;
  double variance = (sig_sq / n) - ((sig / n) * (sig / n));
  double service_rate = 1.0 / (sig / n);
  double arrival_rate = ((double)n) / newest;
  if (arrival_rate >= service_rate) arrival_rate = 0.999 * service_rate;
  return (uint64_t)ceil(0.5 * service_rate * arrival_rate * ((1 / (service_rate * service_rate)) + variance) /
                        (service_rate - arrival_rate));
}
constexpr uint64_t kMg1Exact = 1ull << 53;

struct HTree {
  HQueue* q; HNode* nd; uint64_t min_proc; bool analytical;

  __device__ __forceinline__ uint64_t mg1_delay() const { return mg1_queue_delay(q->n, q->newest, q->sig_sq, q->sig); }
  // ---- sorted interval array nd[0..size) (history_tree and history_list) ----
  __device__ __forceinline__ void l_erase(uint32_t i)
  {
    for (uint32_t j = i + 1; j < q->size; ++j) nd[j - 1] = nd[j];
    q->size--;
  }
  __device__ __forceinline__ void l_insert(uint32_t i, uint64_t a, uint64_t b)   // before position i
  {
    for (uint32_t j = q->size; j > i; --j) nd[j] = nd[j - 1];
    nd[i].first = a; nd[i].second = b;
    q->size++;
  }
  // ---- history_tree: circular sorted list.  The header words live in
  // registers for the request (the queue may sit in LDS or HBM; stores to
  // the interval slots would otherwise force them to be reloaded) ----
  struct TL {
    HNode* nd; uint32_t head, cap, n;
    __device__ __forceinline__ uint32_t ph(uint32_t i) const { const uint32_t j = head + i; return j >= cap ? j - cap : j; }
    __device__ __forceinline__ HNode& iv(uint32_t i) const { return nd[ph(i)]; }
    __device__ __forceinline__ void erase(uint32_t i)
    {
      if (i == 0) { head = ph(1); --n; return; }
      for (uint32_t j = i + 1; j < n; ++j) iv(j - 1) = iv(j);
      --n;
    }
    __device__ __forceinline__ void insert(uint32_t i, uint64_t a, uint64_t b)     // before position i (n < cap)
    {
      for (uint32_t j = n; j > i; --j) iv(j) = iv(j - 1);
      HNode& x = iv(i);
      x.first = a; x.second = b;
      ++n;
    }
    // first fit (searchTree, see above): the last interval starting at or
    // before t if it holds [t, t+p], else the first later one of length >= p
    __device__ __forceinline__ int first_fit(uint64_t t, uint64_t p) const
    {
      int lo = 0, hi = (int)n;
      if (n) { const HNode& l = iv(n - 1); if (l.first <= t) { if (t + p <= l.second) return (int)n - 1; lo = (int)n; } }
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (iv(mid).first <= t) lo = mid + 1; else hi = mid; }
      const int j = lo - 1;
      if (j >= 0 && t + p <= iv(j).second) return j;
      for (int i = j + 1; i < (int)n; ++i) { const HNode& x = iv(i); if (x.second - x.first >= p) return i; }
      return -1;
    }
  };
  __device__ __forceinline__ uint64_t tree_delay(uint64_t t, uint64_t p, uint32_t* err)   // computeQueueDelay (:44-126)
  {
    TL L{nd, q->head, q->max_size, q->size};
    uint64_t qd = 0;
    if (L.n >= L.cap) L.erase(0);                              // prune the min node (:52-56)
    const HNode x0 = L.iv(0);
    if (analytical && x0.first > (t + p)) {
      q->analytical++;
      qd = mg1_delay();
    } else {
      const int i = L.first_fit(t, p);
      if (i < 0) { atomicOr(err, GG_DERR_STATE); }
      else {
        HNode& x = L.iv((uint32_t)i);
        const uint64_t a = x.first, b = x.second;
        if (t >= a) {
          if ((t - a) >= min_proc) {
            if ((b - (t + p)) >= min_proc) L.insert((uint32_t)i + 1, t + p, b);
            L.iv((uint32_t)i).second = t;
          } else if ((b - (t + p)) >= min_proc) {
            x.first = t + p;
          } else {
            L.erase((uint32_t)i);
          }
        } else {
          qd = a - t;
          if ((b - (a + p)) >= min_proc) x.first = a + p;
          else L.erase((uint32_t)i);
        }
      }
    }
    q->head = L.head; q->size = L.n;
    return qd;
  }
  // ---- history_tree on a whole wave (every lane, identical arguments; the
  // image in LDS, max_size <= 128): logical interval i in lane i & 63, slot
  // i >> 6.  The same request as tree_delay: the search is two ballots, an
  // insert / erase a shift of the lanes' registers, the write back one
  // store round of the slots that changed (same circular layout) ----
  __device__ __forceinline__ static uint64_t sh64(uint64_t v, uint32_t src) { return (uint64_t)__shfl((long long)v, (int)src); }
  __device__ __forceinline__ static uint64_t rl64(uint64_t v, uint32_t l)
  {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), (int)l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  }
  __device__ __forceinline__ uint64_t tree_delay_wave(uint64_t t, uint64_t p, uint32_t* err, uint32_t ln)
  {
    const uint32_t cap = q->max_size;
    uint32_t head = q->head, n = q->size;
    if (n >= cap) { head = head + 1 == cap ? 0u : head + 1; --n; }    // prune the min node (:52-56)
    auto phys = [&](uint32_t i) { uint32_t j = head + i; if (j >= cap) j -= cap; if (j >= cap) j -= cap; return j; };
    {
      // the last interval is always [x, UINT64_MAX) (the initial node's end; a
      // request only cuts finite pieces).  A request at t >= x is served there
      // with no delay, and interval 0 starts at or before x, so the M/G/1
      // branch cannot be taken: O(1) on uniform values
      const uint32_t pl = phys(n - 1);
      const HNode last = nd[pl];
      if (last.first <= t) {
        if (t - last.first >= min_proc) {
          nd[pl].second = t;
          nd[phys(n)] = HNode{t + p, last.second};
          ++n;
        } else {
          nd[pl].first = t + p;
        }
        q->head = head; q->size = n;
        wave_sync();
        return 0;
      }
    }
    const bool two = cap > 64;
    uint64_t a0 = 0, b0 = 0, a1 = 0, b1 = 0;
    if (ln < n) { const HNode x = nd[phys(ln)]; a0 = x.first; b0 = x.second; }
    if (two && ln + 64 < n) { const HNode x = nd[phys(ln + 64)]; a1 = x.first; b1 = x.second; }
    uint64_t qd = 0;
    uint32_t ch = n, nn = n;                       // first logical slot that changed, new size
    if (analytical && rl64(a0, 0) > t + p) {
      q->analytical++;
      qd = mg1_delay();
    } else {
      // first fit: j = the last interval starting at or before t
      const bool v0 = ln < n, v1 = ln + 64 < n;
      const uint32_t cnt = (uint32_t)__builtin_popcountll(__ballot(v0 && a0 <= t)) +
                           (uint32_t)__builtin_popcountll(__ballot(v1 && a1 <= t));
      int i = -1;
      if (cnt > 0) {
        const uint32_t j = cnt - 1;
        const uint64_t bj = j < 64 ? rl64(b0, j) : rl64(b1, j - 64);
        if (t + p <= bj) i = (int)j;
      }
      if (i < 0) {
        const uint64_t m0 = __ballot(v0 && ln >= cnt && b0 - a0 >= p);
        const uint64_t m1 = __ballot(v1 && ln + 64 >= cnt && b1 - a1 >= p);
        i = m0 ? (int)__builtin_ctzll(m0) : (m1 ? 64 + (int)__builtin_ctzll(m1) : -1);
      }
      if (i < 0) {
        if (ln == 0) atomicOr(err, GG_DERR_STATE);
      } else {
        const uint32_t ui = (uint32_t)i;
        const uint64_t a = ui < 64 ? rl64(a0, ui) : rl64(a1, ui - 64);
        const uint64_t b = ui < 64 ? rl64(b0, ui) : rl64(b1, ui - 64);
        uint64_t na = a, nb = b;                    // new interval ui (if it stays)
        int op = 0;                                 // 0 modify, 1 insert (t + p, b) after ui, 2 erase ui
        if (t >= a) {
          if ((t - a) >= min_proc) { nb = t; if ((b - (t + p)) >= min_proc) op = 1; }
          else if ((b - (t + p)) >= min_proc) na = t + p;
          else op = 2;
        } else {
          qd = a - t;
          if ((b - (a + p)) >= min_proc) na = a + p; else op = 2;
        }
        ch = ui;
        if (op == 1) {                              // new(k) = old(k - 1) for k > ui + 1
          const uint32_t s = (ln + 63) & 63;
          const uint64_t pa0 = sh64(a0, s), pb0 = sh64(b0, s), pa1 = sh64(a1, s), pb1 = sh64(b1, s);
          if (ln > ui + 1) { a0 = pa0; b0 = pb0; }
          if (ln + 64 > ui + 1) { a1 = ln == 0 ? pa0 : pa1; b1 = ln == 0 ? pb0 : pb1; }
          const uint32_t k = ui + 1;
          if ((k & 63) == ln) { if (k < 64) { a0 = t + p; b0 = b; } else { a1 = t + p; b1 = b; } }
          nn = n + 1;
        } else if (op == 2) {                       // new(k) = old(k + 1) for k >= ui
          const uint32_t s = (ln + 1) & 63;
          const uint64_t na0 = sh64(a0, s), nb0 = sh64(b0, s), na1 = sh64(a1, s), nb1 = sh64(b1, s);
          if (ln >= ui) { a0 = ln == 63 ? na1 : na0; b0 = ln == 63 ? nb1 : nb0; }
          if (ln + 64 >= ui) { a1 = na1; b1 = nb1; }
          nn = n - 1;
        }
        if (op != 2 && (ui & 63) == ln) { if (ui < 64) { a0 = na; b0 = nb; } else { a1 = na; b1 = nb; } }
      }
    }
    if (ln >= ch && ln < nn) nd[phys(ln)] = HNode{a0, b0};
    if (two && ln + 64 >= ch && ln + 64 < nn) nd[phys(ln + 64)] = HNode{a1, b1};
    q->head = head; q->size = nn;
    wave_sync();
    return qd;
  }
  // replace interval i by up to two intervals (in list order).  The list may
  // overgrow by one only here, and then loses its front (the size check after
  // the scan, queue_model_history_list.cc:128-131): done in place.
  __device__ __forceinline__ void l_replace(uint32_t i, bool k1, uint64_t a1, uint64_t b1, bool k2, uint64_t a2, uint64_t b2)
  {
    if (k1 && !k2) { nd[i].first = a1; nd[i].second = b1; return; }
    if (!k1 && k2) { nd[i].first = a2; nd[i].second = b2; return; }
    if (!k1) { l_erase(i); return; }
    if (q->size < q->max_size) {
      for (uint32_t j = q->size; j > i + 1; --j) nd[j] = nd[j - 1];
      nd[i].first = a1; nd[i].second = b1; nd[i + 1].first = a2; nd[i + 1].second = b2;
      q->size++;
    } else if (i == 0) {                        // the first new interval is the front that goes
      nd[0].first = a2; nd[0].second = b2;
    } else {                                    // drop the front: [1, i) moves down by one
      for (uint32_t j = 1; j < i; ++j) nd[j - 1] = nd[j];
      nd[i - 1].first = a1; nd[i - 1].second = b1; nd[i].first = a2; nd[i].second = b2;
    }
  }
  __device__ __forceinline__ uint64_t list_scan(uint64_t t, uint64_t p)       // computeUsingHistoryList
  {
    uint64_t qd = 0;
    const bool inter = q->aux == 0;
    uint32_t i = 0;
    while (i < q->size) {
      const uint64_t a = nd[i].first, b = nd[i].second;
      if (t >= a && t + p <= b) {
        l_replace(i, t - a >= min_proc, a, t, b - (t + p) >= min_proc, t + p, b);
        return qd;
      }
      if (t < a && a + p <= b) {
        qd += a - t;
        l_replace(i, false, 0, 0, b - (a + p) >= min_proc, a + p, b);
        return qd;
      }
      if (inter && t >= a && t < b) {           // pkt_time moves to b, processing_time -= 0 (as the reference)
        if (t - a >= min_proc) { nd[i].second = t; ++i; } else l_erase(i);
        t = b;
      } else if (inter && t < a) {
        l_erase(i);
        qd += a - t;
        p -= b - a;
        t = b;
      } else {
        ++i;
      }
    }
    return qd;
  }
  // ---- basic: MovingAverage<UInt64>::compute over the window words ----
  __device__ __forceinline__ uint64_t mavg(uint64_t x)
  {
    uint64_t* w = reinterpret_cast<uint64_t*>(nd);
    const uint32_t W = hq_window(q->aux), M = W + 1, avg = q->aux >> 16;
    const uint32_t cws = q->back >= q->front ? q->back - q->front : q->back + M - q->front;
    if (avg != GG_MAVG_MEDIAN) {
      if (cws == W) q->mean += (((double)x / cws) - ((double)w[q->front] / cws));
      else q->mean = (q->mean * cws + (double)x) / (double)(cws + 1);
    }
    w[q->back] = x;                             // addToWindow
    q->back = (q->back + 1) % M;
    if (q->back == q->front) q->front = (q->front + 1) % M;
    if (avg == GG_MAVG_MEDIAN) {
      const uint32_t c2 = q->back >= q->front ? q->back - q->front : q->back + M - q->front;
      return w[(q->front + (c2 / 2) % M) % M];
    }
    return (uint64_t)q->mean;
  }
  __device__ __forceinline__ uint64_t basic_delay(uint64_t t, uint64_t p)
  {
    const uint64_t ref = ((q->aux >> 16) == GG_MAVG_NONE) ? t : mavg(t);
    const uint64_t qd = q->qtime > ref ? q->qtime - ref : 0;
    q->qtime = (q->qtime > ref ? q->qtime : ref) + p;
    q->util += p;
    { uint64_t x = ref + qd + p; if (x > q->last_req) q->last_req = x; }
    q->total_req++;
    return qd;
  }

  __device__ __forceinline__ uint64_t delay(uint64_t t, uint64_t p, uint32_t* err)   // computeQueueDelay
  {
    if (q->type == GG_QM_BASIC) return basic_delay(t, p);
    uint64_t qd;
    if (q->type == GG_QM_HISTORY_LIST) {
      if (analytical && (t + p) < nd[0].first) { q->analytical++; qd = mg1_delay(); }
      else qd = list_scan(t, p);
    } else {
      qd = tree_delay(t, p, err);
    }
    mg1_update(t, p, qd, err);
    return qd;
  }
  // computeQueueDelay on a whole wave (every lane, identical arguments, the
  // queue image in LDS): history_tree lane-parallel, the others as delay()
  __device__ __forceinline__ uint64_t delay_w(uint64_t t, uint64_t p, uint32_t* err, uint32_t ln)
  {
    if (q->type != GG_QM_HISTORY_TREE || q->max_size > 128) return delay(t, p, err);
    const uint64_t qd = tree_delay_wave(t, p, err, ln);
    mg1_update(t, p, qd, err);
    return qd;
  }
  __device__ __forceinline__ void mg1_update(uint64_t t, uint64_t p, uint64_t qd, uint32_t* err)
  {
    const uint64_t ss = q->sig_sq, sg = q->sig;
    const uint64_t nn = q->n, nw = q->newest, ut = q->util, lr = q->last_req, tr = q->total_req;
    const uint64_t x = t + qd + p;
    const uint64_t ss2 = ss + p * p;
    if (ss2 >= kMg1Exact || p >= (1ull << 26)) atomicOr(err, GG_DERR_RANGE);
    q->sig_sq = ss2;                                             // QueueModelMG1::updateQueue
    q->sig = sg + p;
    q->n = nn + 1;
    q->newest = x > nw ? x : nw;
    q->util = ut + p;                                            // updateQueueUtilizationCounters
    q->last_req = x > lr ? x : lr;
    q->total_req = tr + 1;
  }

};

// ---------------------------------------------------------------------------
// One history-tree queue held in a wave's registers for a batch of requests
// (every lane calls every method with identical arguments).  Logical interval
// i (< 128 = max_size bound) sits in lane i & 63 of slot i >> 6, so the
// queue's state costs no memory round trip per request: the search is two
// ballots, an insert / erase a one-lane shift of the slots (DPP wave_shr /
// wave_shl), the header and M/G/1 sums are uniform registers.  load / store
// move the image (HQueue + circular node list, any head) in one round each;
// store writes it back with head 0.  Same request as HTree::tree_delay +
// mg1_update (the in-order request, t at or after the start of the last
// interval [x, UINT64_MAX), is the O(1) first branch).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l)
{
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), (int)l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
}
// a wave-uniform 64-bit value into SGPRs (values computed on the vector ALU,
// e.g. FP64, or loaded by an atomic, are otherwise kept in VGPRs)
__device__ __forceinline__ uint64_t rfl64(uint64_t v)
{
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
template <int CTRL> __device__ __forceinline__ uint64_t dpp64(uint64_t v)
{
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
constexpr int kDppWaveShl1 = 0x130;    // lane l <- lane l + 1
constexpr int kDppWaveShr1 = 0x138;    // lane l <- lane l - 1

// lane mask of a 64-bit comparison (one v_cmp into an SGPR pair, no bool
// materialization between compare and ballot)
template <int PRED> __device__ __forceinline__ uint64_t cmp64(uint64_t a, uint64_t b)
{
  return __builtin_amdgcn_uicmpl(a, b, PRED);
}
constexpr int kCmpULE = 37, kCmpUGE = 35, kCmpUGT = 34;     // ICmpInst predicates
__device__ __forceinline__ uint64_t low_lanes(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

struct RegQueue {
  uint64_t a0, b0, a1, b1;             // this lane's intervals of slot 0 / slot 1
  uint32_t sz, cap, ln;
  uint64_t sig_sq, sig, nreq, newest, util, last_req, total_req, anl;
  uint64_t min_proc;
  bool analytical;
  uint32_t n_fast = 0, n_anl = 0, n_gen = 0;   // requests by branch (diagnostics)
  uint32_t errs = 0;                   // GG_DERR_* of the batch, reported by store()
  uint32_t* errp = nullptr;

  __device__ __forceinline__ void load(const HQueue* q, const HNode* nd, uint64_t mp, bool an, uint32_t lane)
  {
    // the header is wave-uniform: into SGPRs (a load from memory the kernel
    // also writes lands in VGPRs, and the size would then steer every request
    // through exec-masked branches)
    ln = lane; min_proc = mp; analytical = an; errs = 0; errp = nullptr;
    sz = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->size);
    cap = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->max_size);
    const uint32_t head = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->head);
    sig_sq = rfl64(q->sig_sq); sig = rfl64(q->sig); nreq = rfl64(q->n); newest = rfl64(q->newest);
    util = rfl64(q->util); last_req = rfl64(q->last_req); total_req = rfl64(q->total_req); anl = rfl64(q->analytical);
    a0 = b0 = a1 = b1 = 0;
    uint32_t j = head + ln; if (j >= cap) j -= cap;
    if (ln < sz) { const HNode x = nd[j]; a0 = x.first; b0 = x.second; }
    j = head + ln + 64; if (j >= cap) j -= cap; if (j >= cap) j -= cap;
    if (ln + 64 < sz) { const HNode x = nd[j]; a1 = x.first; b1 = x.second; }
  }
  // load() with the node loads issued beside the header's instead of behind
  // it: every store() writes the list back from slot 0 (head 0), so a queue
  // only ever served through RegQueue (hq_init starts at head 0) has head 0 at
  // every load, and nodes [0, max_size) are the list in order.  The header is
  // checked when it arrives: a queue another form left at head != 0 takes the
  // dependent load().  One memory round trip instead of two.
  __device__ __forceinline__ void load_h0(const HQueue* q, const HNode* nd, uint32_t max_size, uint64_t mp, bool an,
                                          uint32_t lane)
  {
    HNode x0{0, 0}, x1{0, 0};
    if (lane < max_size) x0 = nd[lane];
    if (lane + 64 < max_size) x1 = nd[lane + 64];
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->head);
    if (h != 0) { load(q, nd, mp, an, lane); return; }
    ln = lane; min_proc = mp; analytical = an; errs = 0; errp = nullptr;
    sz = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->size);
    cap = (uint32_t)__builtin_amdgcn_readfirstlane((int)q->max_size);
    sig_sq = rfl64(q->sig_sq); sig = rfl64(q->sig); nreq = rfl64(q->n); newest = rfl64(q->newest);
    util = rfl64(q->util); last_req = rfl64(q->last_req); total_req = rfl64(q->total_req); anl = rfl64(q->analytical);
    const bool v0 = ln < sz, v1 = ln + 64 < sz;
    a0 = v0 ? x0.first : 0; b0 = v0 ? x0.second : 0;
    a1 = v1 ? x1.first : 0; b1 = v1 ? x1.second : 0;
  }
  // load_h0 in two halves, so that a wave can issue other loads while the
  // queue's are in flight: issue() starts the loads into registers and waits
  // for nothing (the header spread over lanes, one 16-B chunk per lane k <
  // sizeof(HQueue) / 16; the nodes as load_h0 reads them); finish() reads
  // the header's fields out of the lanes, which waits for them, and takes
  // the dependent load() when the list does not start at node 0.
  struct Raw { uint4 hc; HNode x0, x1; };
  __device__ __forceinline__ static Raw issue(const HQueue* q, const HNode* nd, uint32_t max_size, uint32_t lane)
  {
    Raw r;
    r.x0 = HNode{0, 0}; r.x1 = HNode{0, 0}; r.hc = make_uint4(0, 0, 0, 0);
    if (lane < max_size) r.x0 = nd[lane];
    if (lane + 64 < max_size) r.x1 = nd[lane + 64];
    if (lane < sizeof(HQueue) / 16) r.hc = reinterpret_cast<const uint4*>(q)[lane];
    return r;
  }
  template <size_t OFF>
  __device__ __forceinline__ static uint32_t hw32(const uint4& c)
  {
    static_assert(OFF % 4 == 0 && OFF < sizeof(HQueue), "a 32-bit header word");
    constexpr uint32_t w = OFF / 4, k = w & 3u;
    const uint32_t v = k == 0 ? c.x : k == 1 ? c.y : k == 2 ? c.z : c.w;
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(w >> 2));
  }
  template <size_t OFF>
  __device__ __forceinline__ static uint64_t hw64(const uint4& c)
  {
    return ((uint64_t)hw32<OFF + 4>(c) << 32) | hw32<OFF>(c);
  }
  __device__ __forceinline__ void finish(const Raw& r, const HQueue* q, const HNode* nd, uint64_t mp, bool an, uint32_t lane)
  {
    const uint32_t h = hw32<offsetof(HQueue, head)>(r.hc);
    if (h != 0) { load(q, nd, mp, an, lane); return; }
    ln = lane; min_proc = mp; analytical = an; errs = 0; errp = nullptr;
    sz = hw32<offsetof(HQueue, size)>(r.hc);
    cap = hw32<offsetof(HQueue, max_size)>(r.hc);
    sig_sq = hw64<offsetof(HQueue, sig_sq)>(r.hc); sig = hw64<offsetof(HQueue, sig)>(r.hc);
    nreq = hw64<offsetof(HQueue, n)>(r.hc); newest = hw64<offsetof(HQueue, newest)>(r.hc);
    util = hw64<offsetof(HQueue, util)>(r.hc); last_req = hw64<offsetof(HQueue, last_req)>(r.hc);
    total_req = hw64<offsetof(HQueue, total_req)>(r.hc); anl = hw64<offsetof(HQueue, analytical)>(r.hc);
    const bool v0 = ln < sz, v1 = ln + 64 < sz;
    a0 = v0 ? r.x0.first : 0; b0 = v0 ? r.x0.second : 0;
    a1 = v1 ? r.x1.first : 0; b1 = v1 ? r.x1.second : 0;
  }
  __device__ __forceinline__ void store(HQueue* q, HNode* nd) const
  {
    if (errs && errp && ln == 0) atomicOr(errp, errs);
    if (ln < sz) nd[ln] = HNode{a0, b0};
    if (ln + 64 < sz) nd[ln + 64] = HNode{a1, b1};
    q->size = sz; q->head = 0;
    q->sig_sq = sig_sq; q->sig = sig; q->n = nreq; q->newest = newest;
    q->util = util; q->last_req = last_req; q->total_req = total_req; q->analytical = anl;
  }
  // interval i's bounds: both slots read, then a scalar select (no branch)
  __device__ __forceinline__ uint64_t A(uint32_t i) const
  {
    const uint32_t l = i & 63; const uint64_t u = rl64(a0, l), v = rl64(a1, l); return i < 64 ? u : v;
  }
  __device__ __forceinline__ uint64_t B(uint32_t i) const
  {
    const uint32_t l = i & 63; const uint64_t u = rl64(b0, l), v = rl64(b1, l); return i < 64 ? u : v;
  }
  __device__ __forceinline__ void set(uint32_t i, uint64_t a, uint64_t b)
  {
    if ((i & 63) == ln) { if (i < 64) { a0 = a; b0 = b; } else { a1 = a; b1 = b; } }
  }
  // new[x] = old[x - 1] for x > k
  __device__ __forceinline__ void shift_up(uint32_t k)
  {
    const uint64_t ca = rl64(a0, 63), cb = rl64(b0, 63);
    const uint64_t pa0 = dpp64<kDppWaveShr1>(a0), pb0 = dpp64<kDppWaveShr1>(b0);
    const uint64_t pa1 = dpp64<kDppWaveShr1>(a1), pb1 = dpp64<kDppWaveShr1>(b1);
    if (ln > k) { a0 = pa0; b0 = pb0; }
    if (ln + 64 > k) { a1 = ln == 0 ? ca : pa1; b1 = ln == 0 ? cb : pb1; }
  }
  // new[x] = old[x + 1] for x >= k
  __device__ __forceinline__ void shift_down(uint32_t k)
  {
    const uint64_t ca = rl64(a1, 0), cb = rl64(b1, 0);
    const uint64_t na0 = dpp64<kDppWaveShl1>(a0), nb0 = dpp64<kDppWaveShl1>(b0);
    const uint64_t na1 = dpp64<kDppWaveShl1>(a1), nb1 = dpp64<kDppWaveShl1>(b1);
    if (ln >= k) { a0 = ln == 63 ? ca : na0; b0 = ln == 63 ? cb : nb0; }
    if (ln + 64 >= k) { a1 = na1; b1 = nb1; }
  }
  // computeQueueDelay (queue_model_history_tree.cc:44-126) + QueueModelMG1::updateQueue.
  // TAIL: also the O(1) branch for requests served by the last two intervals
  // (in-order streams: SELF / injection ports); the walkers' requests land
  // mid-list 84 % of the time and skip that check (TAIL = false: the general
  // search serves those requests too, with the same result).
  template <bool TAIL = true>
  __device__ __forceinline__ uint64_t request(uint64_t t, uint64_t p, uint32_t* err)
  {
    errp = err;
    if (sz >= cap) { shift_down(0); --sz; }                          // prune the min node (:52-56)
    uint64_t qd = 0;
    const uint64_t la = A(sz - 1), lb = B(sz - 1);
    if (la <= t && t + p <= lb && lb - (t + p) >= min_proc) {        // the last interval: no search, no delay
      ++n_fast;
      if (t - la >= min_proc) { set(sz - 1, la, t); set(sz, t + p, lb); ++sz; }
      else set(sz - 1, t + p, lb);
    } else if (TAIL && sz >= 2 && t < la && t >= A(sz - 2)) {
      // the tail: interval sz-2 is the last one starting at or before t (and
      // interval 0 starts before t: no M/G/1).  Either [t, t+p] fits in it, or
      // the first later interval long enough is the last one (unbounded)
      ++n_fast;
      const uint32_t i2 = sz - 2, i1 = sz - 1;
      const uint64_t a2 = A(i2), b2 = B(i2);
      if (t + p <= b2) {
        if (t - a2 >= min_proc) {
          if (b2 - (t + p) >= min_proc) { set(i1 + 1, la, lb); set(i1, t + p, b2); ++sz; }
          set(i2, a2, t);
        } else if (b2 - (t + p) >= min_proc) {
          set(i2, t + p, b2);
        } else {
          set(i2, la, lb); --sz;                                       // erase interval sz-2
        }
      } else {
        qd = la - t;                                                   // queued behind the busy period
        if (lb - (la + p) >= min_proc) set(i1, la + p, lb);
        else --sz;                                                     // erase the last interval
      }
    } else if (analytical && A(0) > t + p) {
      ++anl; ++n_anl;
      qd = mg1_queue_delay(nreq, newest, sig_sq, sig);
    } else {
      ++n_gen;
      // fit: a <= t && t + p <= b — at most one interval (the intervals are
      // disjoint and sorted: any earlier one ends before the last start <= t),
      // the last one starting at or before t; else the first later one
      // (a > t) with b - a >= p.  Lane masks straight from the compares.
      const uint64_t tp = t + p;
      const uint64_t v0 = low_lanes(sz), v1 = sz > 64 ? low_lanes(sz - 64) : 0ull;
      const uint64_t le0 = cmp64<kCmpULE>(a0, t) & v0, le1 = cmp64<kCmpULE>(a1, t) & v1;
      const uint64_t f0 = le0 & cmp64<kCmpUGE>(b0, tp), f1 = le1 & cmp64<kCmpUGE>(b1, tp);
      const uint64_t l0 = ~le0 & v0 & cmp64<kCmpUGE>(b0 - a0, p), l1 = ~le1 & v1 & cmp64<kCmpUGE>(b1 - a1, p);
      const bool fit = (f0 | f1) != 0;
      const uint64_t m0 = fit ? f0 : l0, m1 = fit ? f1 : l1;
      const int i = m0 ? (int)__builtin_ctzll(m0) : (m1 ? 64 + (int)__builtin_ctzll(m1) : -1);
      if (i < 0) {
        errs |= GG_DERR_STATE;
      } else {
        const uint32_t ui = (uint32_t)i;
        const uint64_t a = A(ui), b = B(ui);
        if (t >= a) {
          if (t - a >= min_proc) {
            if (b - (t + p) >= min_proc) { shift_up(ui + 1); set(ui + 1, t + p, b); ++sz; }
            set(ui, a, t);
          } else if (b - (t + p) >= min_proc) {
            set(ui, t + p, b);
          } else {
            shift_down(ui); --sz;
          }
        } else {
          qd = a - t;
          if (b - (a + p) >= min_proc) set(ui, a + p, b);
          else { shift_down(ui); --sz; }
        }
      }
    }
    sig_sq += p * p;                                                 // QueueModelMG1::updateQueue
    sig += p;
    if (sig_sq >= kMg1Exact || p >= (1ull << 26)) errs |= GG_DERR_RANGE;
    ++nreq;
    const uint64_t x = t + qd + p;
    newest = x > newest ? x : newest;
    util += p;                                                       // updateQueueUtilizationCounters
    last_req = x > last_req ? x : last_req;
    ++total_req;
    return qd;
  }
  // The same request with the delay handed to pub(qd) as soon as it is
  // known, before the interval list and the M/G/1 sums are updated: a
  // pipeline stage forwards its packet first and does the bookkeeping while
  // the next stage runs (this queue's next request comes from the same wave,
  // after it).  One vector search serves every case (no last-interval
  // pre-check: the walkers' requests land mid-list, and the last interval
  // [x, inf) is found by the same compares): the interval holding t fits
  // [t, t+p] -> no delay, published after two compares; otherwise either the
  // analytical branch (interval 0 starts after t + p; never with a fit, whose
  // interval starts at or before t) or the first later interval long enough.
  // Uniform values are kept scalar (readfirstlane) so a loop around it
  // carries them in SGPRs.
  __device__ __forceinline__ uint64_t rd64(uint64_t v) const { return rfl64(v); }
  __device__ __forceinline__ uint64_t A1(uint32_t i) const { return i < 64 ? rl64(a0, i) : rl64(a1, i - 64); }
  __device__ __forceinline__ uint64_t B1(uint32_t i) const { return i < 64 ? rl64(b0, i) : rl64(b1, i - 64); }
  template <class Pub>
  __device__ __forceinline__ uint64_t request_pub(uint64_t t, uint64_t p, Pub&& pub)
  {
    if (sz >= cap) { shift_down(0); --sz; }                          // prune the min node (:52-56)
    uint64_t qd = 0;
    const uint64_t tp = t + p;
    const uint64_t v0 = low_lanes(sz), v1 = sz > 64 ? low_lanes(sz - 64) : 0ull;
    const uint64_t le0 = cmp64<kCmpULE>(a0, t) & v0, le1 = cmp64<kCmpULE>(a1, t) & v1;
    const uint64_t f0 = le0 & cmp64<kCmpUGE>(b0, tp), f1 = le1 & cmp64<kCmpUGE>(b1, tp);
    if (f0 | f1) {                                                   // a <= t, t + p <= b: no delay
      pub(0ull);
      ++n_gen;
      const uint32_t ui = f0 ? (uint32_t)__builtin_ctzll(f0) : 64u + (uint32_t)__builtin_ctzll(f1);
      const uint64_t a = A1(ui), b = B1(ui);
      if (t - a >= min_proc) {
        if (b - tp >= min_proc) { shift_up(ui + 1); set(ui + 1, tp, b); ++sz; }
        set(ui, a, t);
      } else if (b - tp >= min_proc) {
        set(ui, tp, b);
      } else {
        shift_down(ui); --sz;
      }
    } else if (analytical && (cmp64<kCmpUGT>(a0, tp) & 1ull)) {     // interval 0 starts after t + p
      qd = mg1_queue_delay(nreq, newest, sig_sq, sig);
      pub(qd);
      ++anl; ++n_anl;
    } else {                                                         // the first later interval long enough
      ++n_gen;
      const uint64_t m0 = ~le0 & v0 & cmp64<kCmpUGE>(b0 - a0, p);
      const uint64_t m1 = ~le1 & v1 & cmp64<kCmpUGE>(b1 - a1, p);
      if ((m0 | m1) == 0) {
        pub(0ull);
        errs |= GG_DERR_STATE;
      } else {
        const uint32_t ui = m0 ? (uint32_t)__builtin_ctzll(m0) : 64u + (uint32_t)__builtin_ctzll(m1);
        const uint64_t a = A1(ui);
        qd = a - t;
        pub(qd);
        const uint64_t b = B1(ui);
        if (b - (a + p) >= min_proc) set(ui, a + p, b);
        else { shift_down(ui); --sz; }
      }
    }
    sig_sq = rd64(sig_sq + p * p);                                   // QueueModelMG1::updateQueue
    sig = rd64(sig + p);
    if (sig_sq >= kMg1Exact || p >= (1ull << 26)) errs |= GG_DERR_RANGE;
    nreq = rd64(nreq + 1);
    const uint64_t x = t + qd + p;
    newest = rd64(x > newest ? x : newest);
    util = rd64(util + p);                                           // updateQueueUtilizationCounters
    last_req = rd64(x > last_req ? x : last_req);
    total_req = rd64(total_req + 1);
    anl = rd64(anl);
    sz = (uint32_t)__builtin_amdgcn_readfirstlane((int)sz);
    return qd;
  }
};

// Latency::toPicosec / Time::toCycles (time_types.h:81-109), double and ceil.
// At 1 GHz (every clock domain of carbon_sim.cfg) both are exact integer
// maps below 2^52 ps: 1000 * cycles / 1.0 is exact, and the correctly
// rounded ps / 1000.0 of a non-multiple of 1000 stays more than 2^-11 away
// from an integer, so its ceil is (ps + 999) / 1000.  Integer arithmetic
// there, the double formula elsewhere.
__device__ __forceinline__ uint64_t lat_to_ps(uint64_t cycles, double f)
{
  if (f == 1.0 && cycles < (1ull << 42)) return 1000 * cycles;
  return (uint64_t)ceil(((double)1000 * cycles) / f);
}
__device__ __forceinline__ uint64_t time_to_cycles(uint64_t ps, double f)
{
  if (f == 1.0 && ps < (1ull << 52)) return (ps + 999) / 1000;
  return (uint64_t)ceil(((double)ps * f) / 1.0e3);
}

struct NocParams {
  uint32_t tiles, w, h, flit_width, router_delay, link_delay, qm, analytical, max_size, net_model;
  uint32_t qtype, qaux;                 // router queue model (GG_QM_*) and its hq_aux parameter
  double f;
};

__device__ __forceinline__ uint64_t nflits(const NocParams& P, uint32_t bits)
{
  return (bits % P.flit_width == 0) ? bits / P.flit_width : bits / P.flit_width + 1;   // computeNumFlits
}

__device__ __forceinline__ void cadd(uint64_t* c, uint32_t tile, int k, uint64_t v)
{
  if (v) atomicAdd((unsigned long long*)&c[(uint64_t)tile * GG_NUM_NET_COUNTERS + k], (unsigned long long)v);
}


// emesh_hop_counter (network_model_emesh_hop_counter.cc:143-157) / magic
// (network_model_magic.cc:5-21) for one packet, with the sender / receiver
// counters and processReceivedPacket's serialization (network_model.cc:142-150).
// Returns the time the packet is handed to the receiver; zl = zero-load part.
__device__ __forceinline__ uint64_t route_closed_form(const NocParams& P, uint32_t s, uint32_t d, uint32_t bits,
                                                      uint64_t t, uint64_t& zl, uint64_t* ctr)
{
  zl = 0;
  if (s == d) return t;                           // processCornerCases: self-sends cost nothing
  if (P.net_model == GG_NET_MAGIC) {
    cadd(ctr, s, GG_NC_PACKETS_SENT, 1); cadd(ctr, s, GG_NC_BITS_SENT, bits);
    const uint64_t l = lat_to_ps(1, P.f);
    t += l; zl += l;
    cadd(ctr, d, GG_NC_PACKETS_RECEIVED, 1); cadd(ctr, d, GG_NC_BITS_RECEIVED, bits);
    cadd(ctr, d, GG_NC_TOTAL_LATENCY_PS, zl);
    return t;
  }
  const uint64_t nf = nflits(P, bits);
  cadd(ctr, s, GG_NC_PACKETS_SENT, 1); cadd(ctr, s, GG_NC_FLITS_SENT, nf); cadd(ctr, s, GG_NC_BITS_SENT, bits);
  const int sx = (int)(s % P.w), sy = (int)(s / P.w), dx = (int)(d % P.w), dy = (int)(d / P.w);
  const uint64_t hops = (uint64_t)(abs(sx - dx) + abs(sy - dy));
  const uint64_t lat = lat_to_ps(hops * ((uint64_t)P.router_delay + P.link_delay), P.f);
  t += lat; zl += lat;
  cadd(ctr, s, GG_NC_BUFFER_WRITES, nf * hops); cadd(ctr, s, GG_NC_BUFFER_READS, nf * hops);
  cadd(ctr, s, GG_NC_SWITCH_ALLOC, hops); cadd(ctr, s, GG_NC_CROSSBAR, nf * hops);
  cadd(ctr, s, GG_NC_LINK_TRAVERSALS, nf * hops);
  const uint64_t ser = lat_to_ps(nf, P.f);
  t += ser; zl += ser;
  cadd(ctr, d, GG_NC_PACKETS_RECEIVED, 1); cadd(ctr, d, GG_NC_FLITS_RECEIVED, nf);
  cadd(ctr, d, GG_NC_BITS_RECEIVED, bits); cadd(ctr, d, GG_NC_TOTAL_LATENCY_PS, zl);
  return t;
}

}  // namespace gg

// accessors of the NoC state (gg_noc.hip) for the coherent path
gg::NocParams gg_noc_params(gg_ctx* ctx);
uint64_t* gg_noc_ctr(gg_ctx* ctx);
// hop-by-hop stage pipeline over up to `cap` packets (*n_dev of them when given);
// khi / klo: canonical tie-break keys (NULL: the packet index)
gg_status gg_noc_hbh(gg_ctx* ctx, const uint32_t* src, const uint32_t* dst, const uint32_t* len, const uint64_t* t0,
                     const uint64_t* khi, const uint64_t* klo, uint64_t cap, const uint32_t* n_dev, hipStream_t s);
const uint64_t* gg_noc_packet_times(gg_ctx* ctx);   // arrival times of the last pipeline run
// the router queues [tile * 6 + port] (ports 0..4 mesh SELF LEFT RIGHT DOWN UP, 5 injection)
void gg_noc_queues(gg_ctx* ctx, gg::HQueue** q, gg::HNode** nd);
