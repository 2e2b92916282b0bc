// gg_round.hip — the lax-barrier round of the coherent mode over ranks, with
// RCCL over xGMI: one process per GPU, each owning a block of logical shards.
//
// Reference: every process exchanges ShmemMsgs over its transport in real
// time (common/transport/socktransport.cc:401-448) and the clocks meet at the
// lax barrier once per quantum (clock_skew_management_schemes/
// lax_barrier_sync_client.cc:31-69, lax_barrier_sync_server.cc:57-160).
// Here the records that cross a rank's shards are held to the quantum
// boundary and exchanged there in ONE grouped send / receive of
// fixed-capacity per-peer slots (a header record carries the count, so no
// count exchange precedes the data), followed by the status all-reduces and
// the import — all enqueued on the context's stream, then one host sync.
// Only a quantum whose records overflow a slot takes a second, sized round.
//
// Failure is decided collectively: a rank whose quantum or export failed still
// posts every send / receive and all-reduce (with its error flag in the
// max-reduced status word), the imports are skipped on the device when the
// reduced flag is set, and every rank returns the error together — no peer is
// left blocked inside RCCL.
#include "gg_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

constexpr uint64_t kSlotDefault = 1024;   // records per peer and quantum sent in the fixed round (64 KB)
constexpr int kDv = 8;                    // status words: sent, active, blocked | err, max slot count | min next

struct RoundBufs {
  gg_cmsg* send = nullptr; gg_cmsg* recv = nullptr;   // [world][1 + region] each
  uint64_t* dv = nullptr;                             // [kDv + 2 * world]: status, send counts, recv counts
  uint64_t* host = nullptr;                           // pinned copy of dv
  uint64_t region = 0; int world = 0;
};

#define GG_NCCL(x)                                                                                         \
  do {                                                                                                     \
    ncclResult_t r_ = (x);                                                                                 \
    if (r_ != ncclSuccess) return gg_fail(GG_ERR_STATE, "%s: %s", #x, ncclGetErrorString(r_));              \
  } while (0)

void bufs_free(void* p)
{
  RoundBufs* b = static_cast<RoundBufs*>(p);
  hipFree(b->send); hipFree(b->recv); hipFree(b->dv); hipHostFree(b->host);
  delete b;
}

gg_status bufs_for(gg_ctx* ctx, RoundBufs*& B, int world, uint64_t region)
{
  B = static_cast<RoundBufs*>(gg_round_state(ctx));
  if (B && B->world == world && B->region >= region) return GG_OK;
  if (B) bufs_free(B);
  gg_round_state_set(ctx, nullptr, nullptr);
  B = new RoundBufs();
  B->region = region; B->world = world;
  gg_round_state_set(ctx, B, bufs_free);
  const size_t slots = (size_t)world * (region + 1);
  GG_HIP(hipMalloc((void**)&B->send, sizeof(gg_cmsg) * slots));
  GG_HIP(hipMalloc((void**)&B->recv, sizeof(gg_cmsg) * slots));
  GG_HIP(hipMalloc((void**)&B->dv, sizeof(uint64_t) * (kDv + 2 * (size_t)world)));
  GG_HIP(hipHostMalloc((void**)&B->host, sizeof(uint64_t) * (kDv + 2 * (size_t)world)));
  return GG_OK;
}

// the slot counts (header word 0) of the send and the received slots
__global__ void k_slot_counts(const gg_cmsg* send, const gg_cmsg* recv, uint32_t world, uint64_t region, uint64_t* out)
{
  for (uint32_t r = threadIdx.x; r < world; r += blockDim.x) {
    out[r] = send[(size_t)r * (region + 1)].addr;
    out[world + r] = recv[(size_t)r * (region + 1)].addr;
  }
}

uint64_t slot_records(uint64_t region)
{
  const char* e = getenv("GG_ROUND_SLOT");          // test knob: a small slot forces the overflow round
  uint64_t v = e ? strtoull(e, nullptr, 10) : kSlotDefault;
  return std::max<uint64_t>(1, std::min(v, region));
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
  // The checks above and these two return before any RCCL call: they depend
  // only on arguments and on gg_coherent_begin having run, which every rank of
  // one program gets identically, so they fail on every rank at once (the
  // send-buffer allocation of the first round is the one rank-local failure
  // that cannot be turned into the round's error flag: there is no buffer).
  const uint64_t region = gg_coherent_msg_cap(ctx);
  if (!region) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  RoundBufs* B = nullptr;
  if (gg_status st = bufs_for(ctx, B, W, region)) return st;
  const uint64_t slot = slot_records(region);
  const size_t sbytes = sizeof(gg_cmsg) * (slot + 1);

  // the quantum and the export; a failure (a wrong stream included) turns into
  // the error flag of the round, which every rank still takes part in
  uint32_t herr = 0;
  std::string emsg;
  gg_status est = GG_OK;
  const bool wrong_stream = s != ctx->last_stream;        // the context's kernels run on last_stream
  if (wrong_stream) est = gg_fail(GG_ERR_INVALID, "gg_round_exchange needs the stream of gg_coherent_begin");
  if (est || (est = gg_coh_quantum_async(ctx, q)) || (est = gg_coh_export_slots(ctx, B->send, (uint32_t)W, per, region))) {
    herr = GG_DERR_STATE;
    emsg = gg_last_error();
    (void)hipMemsetAsync(B->send, 0, sizeof(gg_cmsg) * (size_t)W * (region + 1), s);   // nothing to send
  }
  if (gg_status st = gg_coh_round_status(ctx, B->send, (uint32_t)W, region, herr, B->dv)) return st;
  if (wrong_stream) GG_HIP(hipStreamSynchronize(ctx->last_stream));   // the status words before RCCL reads them on s
  // ONE group: every peer's fixed slot; then the status all-reduces
  GG_NCCL(ncclGroupStart());
  for (int r = 0; r < W; ++r) {
    GG_NCCL(ncclSend(B->send + (size_t)r * (region + 1), sbytes, ncclUint8, r, comm, s));
    GG_NCCL(ncclRecv(B->recv + (size_t)r * (region + 1), sbytes, ncclUint8, r, comm, s));
  }
  GG_NCCL(ncclGroupEnd());
  GG_NCCL(ncclGroupStart());
  GG_NCCL(ncclAllReduce(B->dv, B->dv, 3, ncclUint64, ncclSum, comm, s));
  GG_NCCL(ncclAllReduce(B->dv + 3, B->dv + 3, 2, ncclUint64, ncclMax, comm, s));
  GG_NCCL(ncclAllReduce(B->dv + 5, B->dv + 5, 1, ncclUint64, ncclMin, comm, s));
  GG_NCCL(ncclGroupEnd());
  if (wrong_stream) {                                      // this rank failed: nothing to import
    GG_HIP(hipStreamSynchronize(s));
    return gg_fail(est, "%s", emsg.c_str());
  }
  // the received records (skipped on the device when any rank failed), the counts, one sync
  if (gg_status st = gg_coh_import_slots(ctx, B->recv, (uint32_t)W, region, 0, slot, true, B->dv + 3)) return st;
  hipLaunchKernelGGL(k_slot_counts, dim3(1), dim3(64), 0, s, B->send, B->recv, (uint32_t)W, region, B->dv + kDv);
  GG_HIP(hipMemcpyAsync(B->host, B->dv, sizeof(uint64_t) * (kDv + 2 * (size_t)W), hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  const uint64_t* h = B->host;
  if (h[3]) {
    if (herr) return gg_fail(est ? est : GG_ERR_STATE, "%s", emsg.c_str());
    if (gg_status st = gg_coh_check(ctx)) return st;
    return gg_fail(GG_ERR_STATE, "quantum %llu failed on another rank", (unsigned long long)q);
  }
  // a slot overflowed somewhere: every rank takes the sized round (the counts are known on both sides now)
  if (h[4] > slot) {
    const uint64_t* sc = h + kDv;
    const uint64_t* rc = h + kDv + W;
    GG_NCCL(ncclGroupStart());
    for (int r = 0; r < W; ++r) {
      const size_t o = (size_t)r * (region + 1) + 1 + slot;
      if (sc[r] > slot) GG_NCCL(ncclSend(B->send + o, sizeof(gg_cmsg) * (sc[r] - slot), ncclUint8, r, comm, s));
      if (rc[r] > slot) GG_NCCL(ncclRecv(B->recv + o, sizeof(gg_cmsg) * (rc[r] - slot), ncclUint8, r, comm, s));
    }
    GG_NCCL(ncclGroupEnd());
    if (gg_status st = gg_coh_import_slots(ctx, B->recv, (uint32_t)W, region, slot, region, false, nullptr)) return st;
    GG_HIP(hipStreamSynchronize(s));
  }
  const uint64_t msgs = h[0], active = h[1], blocked = h[2], mn = h[5];
  const uint64_t qps = (uint64_t)c.quantum_ns * 1000ull;
  *done = 0;
  if (active == 0 && msgs == 0) { *done = 1; *next_q = q; return gg_coh_check(ctx); }
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
