// gg_round.hip — the lax-barrier round of the coherent mode over ranks, with
// RCCL over xGMI: one process per GPU, each owning a block of logical shards.
//
// Reference: every process exchanges ShmemMsgs over its transport in real
// time (common/transport/socktransport.cc) and the clocks meet at the lax
// barrier once per quantum (clock_skew_management_schemes/
// lax_barrier_sync_client.cc:31-69, lax_barrier_sync_server.cc:57-160).
// Here the records that cross a rank's shards are held to the quantum
// boundary and exchanged there in one grouped send / receive
// per peer; the status (records in flight, active / blocked tiles, earliest
// next start) is all-reduced, and every rank derives the same next quantum
// (the rule of oracle_coh_run and graphite_amd.coherent.next_quantum).
#include "gg_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <vector>

namespace {

struct RoundBufs {
  gg_cmsg* send = nullptr; gg_cmsg* recv = nullptr; uint64_t* cnt = nullptr;   // cnt: [W] send, [W] recv, [4] status
  uint64_t cap = 0; int world = 0;
};

#define GG_NCCL(x)                                                                                         \
  do {                                                                                                     \
    ncclResult_t r_ = (x);                                                                                 \
    if (r_ != ncclSuccess) return gg_fail(GG_ERR_STATE, "%s: %s", #x, ncclGetErrorString(r_));              \
  } while (0)

gg_status bufs_for(gg_ctx* ctx, RoundBufs*& B, int world, uint64_t cap)
{
  B = static_cast<RoundBufs*>(gg_round_state(ctx));
  if (B && B->world == world && B->cap >= cap) return GG_OK;
  if (B) { hipFree(B->send); hipFree(B->recv); hipFree(B->cnt); delete B; }
  B = new RoundBufs();
  B->cap = cap; B->world = world;
  GG_HIP(hipMalloc((void**)&B->send, sizeof(gg_cmsg) * cap));
  GG_HIP(hipMalloc((void**)&B->recv, sizeof(gg_cmsg) * cap));
  GG_HIP(hipMalloc((void**)&B->cnt, sizeof(uint64_t) * (2 * (size_t)world + 4)));
  gg_round_state_set(ctx, B, [](void* p) {
    RoundBufs* b = static_cast<RoundBufs*>(p);
    hipFree(b->send); hipFree(b->recv); hipFree(b->cnt);
    delete b;
  });
  return GG_OK;
}

}  // namespace

gg_status gg_round_exchange(gg_ctx* ctx, void* nccl_comm, void* stream, uint64_t q, uint64_t* next_q, int* done)
{
  if (!ctx || !nccl_comm || !next_q || !done) return gg_fail(GG_ERR_INVALID, "NULL argument");
  ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
  int W = 0, R = 0;
  GG_NCCL(ncclCommCount(comm, &W));
  GG_NCCL(ncclCommUserRank(comm, &R));
  const gg_config& c = ctx->cfg;
  const uint32_t K = c.num_shards ? c.num_shards : 1;
  if (K % (uint32_t)W) return gg_fail(GG_ERR_INVALID, "%u logical shards do not split over %d ranks", K, W);
  const uint32_t per = K / (uint32_t)W;
  const uint32_t k1 = c.shard_end ? c.shard_end : K;
  if (c.shard_begin != (uint32_t)R * per || k1 != ((uint32_t)R + 1) * per)
    return gg_fail(GG_ERR_INVALID, "rank %d must own shards [%u, %u), the context owns [%u, %u)", R, R * per,
                   (R + 1) * per, c.shard_begin, k1);
  hipSetDevice(ctx->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t cap = gg_coherent_msg_cap(ctx);
  if (!cap) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  RoundBufs* B = nullptr;
  if (gg_status st = bufs_for(ctx, B, W, cap)) return st;

  gg_coherent_status st;
  if (gg_status e = gg_coherent_quantum(ctx, q, &st)) return e;
  std::vector<uint64_t> per_shard(K, 0);
  if (gg_status e = gg_coherent_export(ctx, B->send, B->cap, per_shard.data())) return e;
  std::vector<uint64_t> h(2 * (size_t)W + 4, 0);
  uint64_t sent = 0;
  for (int r = 0; r < W; ++r)
    for (uint32_t k = r * per; k < (r + 1) * per; ++k) { h[r] += per_shard[k]; sent += per_shard[k]; }
  // counts, then the records (grouped by destination rank: export orders them by shard)
  GG_HIP(hipMemcpyAsync(B->cnt, h.data(), sizeof(uint64_t) * W, hipMemcpyHostToDevice, s));
  GG_NCCL(ncclGroupStart());
  for (int r = 0; r < W; ++r) {
    GG_NCCL(ncclSend(B->cnt + r, 1, ncclUint64, r, comm, s));
    GG_NCCL(ncclRecv(B->cnt + W + r, 1, ncclUint64, r, comm, s));
  }
  GG_NCCL(ncclGroupEnd());
  GG_HIP(hipMemcpyAsync(h.data() + W, B->cnt + W, sizeof(uint64_t) * W, hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  uint64_t total = 0;
  for (int r = 0; r < W; ++r) total += h[W + r];
  if (total > B->cap) return gg_fail(GG_ERR_UNSUPPORTED, "%llu records arrive, the round buffer holds %llu",
                                     (unsigned long long)total, (unsigned long long)B->cap);
  uint64_t so = 0, ro = 0;
  GG_NCCL(ncclGroupStart());
  for (int r = 0; r < W; ++r) {
    if (h[r]) GG_NCCL(ncclSend(B->send + so, h[r] * sizeof(gg_cmsg), ncclUint8, r, comm, s));
    if (h[W + r]) GG_NCCL(ncclRecv(B->recv + ro, h[W + r] * sizeof(gg_cmsg), ncclUint8, r, comm, s));
    so += h[r]; ro += h[W + r];
  }
  GG_NCCL(ncclGroupEnd());
  GG_HIP(hipStreamSynchronize(s));
  if (total) if (gg_status e = gg_coherent_import(ctx, B->recv, total)) return e;
  // status over ranks: sums of (records in flight, active, blocked), min of the next start
  uint64_t sum[3] = {sent, st.active_tiles, st.blocked_tiles}, mn = st.min_next_ps;
  uint64_t* dv = B->cnt + 2 * W;
  GG_HIP(hipMemcpyAsync(dv, sum, sizeof(sum), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemcpyAsync(dv + 3, &mn, sizeof(mn), hipMemcpyHostToDevice, s));
  GG_NCCL(ncclGroupStart());
  GG_NCCL(ncclAllReduce(dv, dv, 3, ncclUint64, ncclSum, comm, s));
  GG_NCCL(ncclAllReduce(dv + 3, dv + 3, 1, ncclUint64, ncclMin, comm, s));
  GG_NCCL(ncclGroupEnd());
  GG_HIP(hipMemcpyAsync(sum, dv, sizeof(sum), hipMemcpyDeviceToHost, s));
  GG_HIP(hipMemcpyAsync(&mn, dv + 3, sizeof(mn), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  const uint64_t msgs = sum[0], active = sum[1], blocked = sum[2];
  const uint64_t qps = (uint64_t)c.quantum_ns * 1000ull;
  *done = 0;
  if (active == 0 && msgs == 0) { *done = 1; *next_q = q; return GG_OK; }
  if (msgs == 0 && blocked != 0) return gg_fail(GG_ERR_STATE, "coherent run deadlocked: tiles blocked with no message in flight");
  *next_q = (msgs == 0) ? std::max<uint64_t>(q + 1, mn / qps) : q + 1;
  return GG_OK;
}

gg_status gg_coherent_run_ranks(gg_ctx* ctx, void* nccl_comm, const gg_trace* tr, uint64_t* access_out_dev, void* stream)
{
  if (gg_status e = gg_coherent_begin(ctx, tr, access_out_dev, stream)) return e;
  uint64_t q = 0;
  for (;;) {
    uint64_t nq = 0;
    int done = 0;
    if (gg_status e = gg_round_exchange(ctx, nccl_comm, stream, q, &nq, &done)) return e;
    if (done) return GG_OK;
    q = nq;
  }
}
