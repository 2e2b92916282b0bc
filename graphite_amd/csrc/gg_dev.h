// gg_dev.h — device-side building blocks shared by the NoC (gg_noc.hip) and
// coherent (gg_coherent.hip) paths: the QueueModelHistoryTree restatement,
// the time conversions and the closed-form EMesh routes.
#pragma once
#include "gg_internal.h"

namespace gg {

// ---------------------------------------------------------------------------
// Queue models (QueueModel::create, queue_model.cc:19-39).  One storage
// layout for all three: HQueue + max_size HNode + max_size int16 free list.
//   history_tree (interval_tree.cc:40-394 + queue_model_history_tree.cc:44-167):
//     AVL nodes + free list;
//   history_list (queue_model_history_list.cc:40-134): the free-interval
//     list as nd[0..size) in list order (first/second);
//   basic (queue_model_basic.cc:34-61): the MovingAverage window
//     (moving_average.h, window + 1 slots) as raw u64 words over nd[].
// ---------------------------------------------------------------------------
struct HNode { uint64_t first, second; int16_t parent, left, right, height; };
struct HQueue {
  int32_t root; uint32_t size; int32_t free_tail; uint32_t max_size;
  double sig_sq, sig; uint64_t n, newest;          // QueueModelMG1
  uint64_t analytical;                              // _total_requests_using_analytical_model
  uint64_t util, last_req, total_req;               // QueueModel utilization counters
  uint32_t type, aux;                               // GG_QM_*; list: no-interleaving flag; basic: basic_moving_avg
  uint32_t front, back;                             // basic: ModuloNum window ends (modulo window + 1)
  double mean;                                      // basic: MovingArithmeticMean::_arithmetic_mean
  uint64_t qtime;                                   // basic: QueueModelBasic::_queue_time
};

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
  if (type == GG_QM_BASIC) {
    if ((aux >> 16) == GG_MAVG_GEOMETRIC_MEAN) return gg_fail(GG_ERR_UNSUPPORTED, "geometric_mean moving average");
    if ((aux >> 16) > GG_MAVG_GEOMETRIC_MEAN) return gg_fail(GG_ERR_INVALID, "unknown moving average type");
    if (hq_window(aux) + 1 > 3 * max_size)
      return gg_fail(GG_ERR_UNSUPPORTED, "moving_avg_window_size + 1 exceeds 3 * max_list_size queue words");
  }
  return GG_OK;
}

// QueueModel{HistoryTree,HistoryList,Basic} constructors on one queue's storage
__device__ inline void hq_init(HQueue* q, HNode* N, int16_t* f, uint32_t max_size, uint32_t type, uint32_t aux)
{
  HQueue Q{};
  Q.max_size = max_size;
  Q.type = type;
  Q.aux = aux;
  if (type == GG_QM_HISTORY_LIST) {
    N[0].first = 0; N[0].second = ~0ull;            // push_back(make_pair(0, UINT64_MAX))
    Q.size = 1;
  } else if (type == GG_QM_BASIC) {
    uint64_t* w = reinterpret_cast<uint64_t*>(N);
    for (uint32_t j = 0; j <= hq_window(aux); ++j) w[j] = 0;   // _num_list.resize(window + 1)
  } else {
    for (uint32_t j = 0; j < max_size; ++j) f[j] = (int16_t)j;  // allocateMemory
    Q.free_tail = (int32_t)max_size - 1;
    const int r = f[Q.free_tail--];                             // allocateNode(PAIR(0, UINT64_MAX))
    N[r].first = 0; N[r].second = ~0ull; N[r].parent = N[r].left = N[r].right = -1; N[r].height = 1;
    Q.root = r; Q.size = 1;
  }
  *q = Q;
}

struct HTree {
  HQueue* q; HNode* nd; int16_t* fl; uint64_t min_proc; bool analytical;

  __device__ __forceinline__ int32_t h(int x) const { return x < 0 ? 0 : nd[x].height; }
  __device__ __forceinline__ void upd_child(int node, int child, int dir)      // updateChildPointer
  {
    if (node < 0) return;
    if (dir == 0) { if (nd[node].first < nd[child].first) nd[node].right = child; else nd[node].left = child; }
    else if (dir == 1) nd[node].left = child;
    else nd[node].right = child;
  }
  __device__ __forceinline__ void upd_parent(int node, int parent)             // updateParentPointer
  {
    if (node >= 0) nd[node].parent = parent;
    if (parent < 0) q->root = node;
  }
  __device__ __forceinline__ bool balanced(int x) const { int d = h(nd[x].left) - h(nd[x].right); return d >= -1 && d <= 1; }
  __device__ __forceinline__ void upd_height(int x) { int a = h(nd[x].left), b = h(nd[x].right); nd[x].height = (int16_t)((a > b ? a : b) + 1); }
  __device__ __forceinline__ void rotate(int y, bool cw)                       // performRotation
  {
    int x;
    if (cw) {
      x = nd[y].left;
      upd_parent(x, nd[y].parent); upd_child(nd[x].parent, x, 0);
      nd[y].left = nd[x].right; upd_parent(nd[y].left, y);
      nd[x].right = (int16_t)y; upd_parent(y, x);
    } else {
      x = nd[y].right;
      upd_parent(x, nd[y].parent); upd_child(nd[x].parent, x, 0);
      nd[y].right = nd[x].left; upd_parent(nd[y].right, y);
      nd[x].left = (int16_t)y; upd_parent(y, x);
    }
    upd_height(y); upd_height(x);
  }
  __device__ __forceinline__ int balance(int z)                                // balanceHeight
  {
    int zl = nd[z].left, zr = nd[z].right;
    bool y_left = h(zl) > h(zr);
    int y = y_left ? zl : zr;
    int yl = nd[y].left, yr = nd[y].right;
    int x; bool x_left;
    if (h(yl) != h(yr)) { x_left = h(yl) > h(yr); x = x_left ? yl : yr; }
    else if (y_left) { x = yl; x_left = true; }
    else { x = yr; x_left = false; }
    if (y_left) {
      if (!x_left) { rotate(y, false); rotate(z, true); return x; }
      rotate(z, true); return y;
    } else {
      if (x_left) { rotate(y, true); rotate(z, false); return x; }
      rotate(z, false); return y;
    }
  }
  __device__ __forceinline__ void rebalance(int r)                             // rebalanceAVLTree
  {
    while (r >= 0) {
      int old = nd[r].height, nr = r;
      if (!balanced(r)) nr = balance(r); else upd_height(r);
      if (nd[nr].height == old) return;
      r = nd[nr].parent;
    }
  }
  __device__ __forceinline__ void insert(int node)                             // insert / insertInTree
  {
    q->size++;
    int r = q->root;
    for (;;) {
      if (nd[node].first < nd[r].first) {
        if (nd[r].left >= 0) r = nd[r].left;
        else { nd[r].left = (int16_t)node; nd[node].parent = (int16_t)r; rebalance(r); return; }
      } else if (nd[node].first > nd[r].first) {
        if (nd[r].right >= 0) r = nd[r].right;
        else { nd[r].right = (int16_t)node; nd[node].parent = (int16_t)r; rebalance(r); return; }
      } else return;   // duplicate key: the reference aborts (LOG_PRINT_ERROR)
    }
  }
  // removeFromTree (interval_tree.cc:322-356) without recursion: the successor
  // of a two-child node has no left child, so its removal is the one-child case
  __device__ __forceinline__ void remove_leafish(int node)
  {
    if (nd[node].left < 0) {
      int p = nd[node].parent;
      if (p >= 0) upd_child(p, nd[node].right, (nd[p].first < nd[node].first) ? 2 : 1);
      upd_parent(nd[node].right, p);
      rebalance(p);
    } else {
      int p = nd[node].parent;
      upd_child(p, nd[node].left, 0);
      upd_parent(nd[node].left, p);
      rebalance(p);
    }
  }
  __device__ __forceinline__ int remove_rec(int node)
  {
    if (nd[node].left < 0 || nd[node].right < 0) { remove_leafish(node); return node; }
    int succ = nd[node].right;
    while (nd[succ].left >= 0) succ = nd[succ].left;           // findMinKeyNode
    remove_leafish(succ);                                      // successor has no left child
    uint64_t f = nd[node].first, s = nd[node].second;          // swap key/interval
    nd[node].first = nd[succ].first; nd[node].second = nd[succ].second;
    nd[succ].first = f; nd[succ].second = s;
    return succ;
  }
  __device__ __forceinline__ int remove(int node) { q->size--; return remove_rec(node); }
  // searchTree (interval_tree.cc:366-394).  The recursion comes back to a
  // node only after searching its LEFT subtree (it descends left only when
  // b < first), so the pending nodes are exactly the ancestors entered through
  // their left child: falling off the tree right after a left descent resumes
  // that node; otherwise the walk climbs parent pointers to the nearest
  // ancestor whose left subtree it is leaving.  No explicit stack (a
  // dynamically indexed array would live in scratch memory).
  __device__ __forceinline__ int search(uint64_t a, uint64_t b) const
  {
    int n = q->root, last = -1;
    bool went_left = false;
    for (;;) {
      if (n < 0) {
        int p;
        if (went_left) {
          p = last;
        } else {
          int c = last;
          for (;;) {
            if (c < 0) return -1;
            p = nd[c].parent;
            if (p < 0) return -1;
            if (nd[p].left == c) break;
            c = p;
          }
        }
        if (a < nd[p].first && (nd[p].second - nd[p].first) >= (b - a)) return p;
        last = p; went_left = false; n = nd[p].right;
        continue;
      }
      if (a >= nd[n].first && b <= nd[n].second) return n;
      if (b < nd[n].first) { last = n; went_left = true; n = nd[n].left; continue; }
      if (a < nd[n].first && (nd[n].second - nd[n].first) >= (b - a)) return n;
      last = n; went_left = false; n = nd[n].right;
    }
  }
  __device__ __forceinline__ int alloc(uint64_t a, uint64_t b)                 // allocateNode
  {
    if (q->free_tail < 0) return -1;
    int i = fl[q->free_tail--];
    nd[i].first = a; nd[i].second = b; nd[i].parent = nd[i].left = nd[i].right = -1; nd[i].height = 1;
    return i;
  }
  __device__ __forceinline__ void release(int i) { fl[++q->free_tail] = (int16_t)i; }
  __device__ __forceinline__ uint64_t mg1_delay() const                         // QueueModelMG1::computeQueueDelay
  {
    if (q->n == 0) return 0;
    double variance = (q->sig_sq / q->n) - ((q->sig / q->n) * (q->sig / q->n));
    double service_rate = 1.0 / (q->sig / q->n);
    double arrival_rate = ((double)q->n) / q->newest;
    if (arrival_rate >= service_rate) arrival_rate = 0.999 * service_rate;
    return (uint64_t)ceil(0.5 * service_rate * arrival_rate * ((1 / (service_rate * service_rate)) + variance) /
                          (service_rate - arrival_rate));
  }
  // ---- history_list: nd[0..size) in list order ----
  __device__ __forceinline__ void l_erase(uint32_t i)
  {
    for (uint32_t j = i + 1; j < q->size; ++j) { nd[j - 1].first = nd[j].first; nd[j - 1].second = nd[j].second; }
    q->size--;
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
      for (uint32_t j = q->size; j > i + 1; --j) { nd[j].first = nd[j - 1].first; nd[j].second = nd[j - 1].second; }
      nd[i].first = a1; nd[i].second = b1; nd[i + 1].first = a2; nd[i + 1].second = b2;
      q->size++;
    } else if (i == 0) {                        // the first new interval is the front that goes
      nd[0].first = a2; nd[0].second = b2;
    } else {                                    // drop the front: [1, i) moves down by one
      for (uint32_t j = 1; j < i; ++j) { nd[j - 1].first = nd[j].first; nd[j - 1].second = nd[j].second; }
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
    uint64_t qd = ~0ull;
    if (q->type == GG_QM_HISTORY_LIST) {
      if (analytical && (t + p) < nd[0].first) { q->analytical++; qd = mg1_delay(); }
      else qd = list_scan(t, p);
      mg1_update(t, p, qd);
      return qd;
    }
    int mn = search(0, 1);
    if (q->size >= q->max_size) release(remove(mn));
    mn = search(0, 1);
    if (analytical && nd[mn].first > (t + p)) {
      q->analytical++;
      qd = mg1_delay();
    } else {
      int node = search(t, t + p);
      if (node < 0) { atomicOr(err, GG_DERR_STATE); return 0; }
      if (t >= nd[node].first) {
        qd = 0;
        if ((t - nd[node].first) >= min_proc) {
          if ((nd[node].second - (t + p)) >= min_proc) {
            int nx = alloc(t + p, nd[node].second);
            if (nx < 0) { atomicOr(err, GG_DERR_STATE); return 0; }
            insert(nx);
          }
          nd[node].second = t;
        } else {
          if ((nd[node].second - (t + p)) >= min_proc) nd[node].first = t + p;
          else release(remove(node));
        }
      } else {
        qd = nd[node].first - t;
        if ((nd[node].second - (nd[node].first + p)) >= min_proc) nd[node].first = nd[node].first + p;
        else release(remove(node));
      }
    }
    mg1_update(t, p, qd);
    return qd;
  }
  __device__ __forceinline__ void mg1_update(uint64_t t, uint64_t p, uint64_t qd)
  {
    q->sig_sq += (double)p * (double)p;                          // QueueModelMG1::updateQueue
    q->sig += (double)p;
    q->n++;
    { uint64_t x = t + qd + p; if (x > q->newest) q->newest = x; }
    q->util += p;                                                // updateQueueUtilizationCounters
    { uint64_t x = t + qd + p; if (x > q->last_req) q->last_req = x; }
    q->total_req++;
  }
};

__device__ __forceinline__ uint64_t lat_to_ps(uint64_t cycles, double f) { return (uint64_t)ceil(((double)1000 * cycles) / f); }
__device__ __forceinline__ uint64_t time_to_cycles(uint64_t ps, double f) { return (uint64_t)ceil(((double)ps * f) / 1.0e3); }

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
