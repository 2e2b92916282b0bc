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
// count exchange precedes the data) and ONE all-gather of the ranks' status
// words.  A round is enqueued whole and synced once: the quantum's steps (a
// batch sized from the quanta before; the launches after its quiet step
// return at once), the tail kernel (status + export, only if the quantum
// finished), the two RCCL groups, the commit + import kernels and the copy
// of the gathered words — every rank reduces them itself.  A rank whose
// quantum had not finished reports not-done: nobody commits or imports, and
// the round runs again with more steps.  Only a quantum whose records
// overflow a slot takes a second, sized round.
//
// Failure is decided collectively: a rank whose quantum or export failed still
// posts every send / receive and the all-gather (with its error flag in its
// status words), the commit and imports are skipped on the device when any
// rank's flag is set, and every rank returns the error together — no peer is
// left blocked inside RCCL.
#include "gg_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kBatchMargin = 3;      // steps launched past the recent quanta's largest (see the round)
constexpr uint64_t kSlotDefault = 1024;   // records per peer and quantum sent in the fixed round (64 KB)

struct RoundBufs {
  gg_cmsg* send = nullptr; gg_cmsg* recv = nullptr;   // [world][1 + region] each
  uint64_t* dv = nullptr;                             // [1 + world][kRoundWords] own, gathered; [2 * world] slot counts
  uint64_t* host = nullptr;                           // pinned copy of the gathered words and counts
  uint64_t region = 0; int world = 0;
  uint32_t steps_hist[4] = {8, 8, 8, 8};              // steps of the last quanta (the batch predictor)
  uint32_t hist_i = 0;
  size_t dv_words() const { return (size_t)(1 + world) * kRoundWords + 2 * (size_t)world; }
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
  GG_HIP(hipMalloc((void**)&B->dv, sizeof(uint64_t) * B->dv_words()));
  GG_HIP(hipHostMalloc((void**)&B->host, sizeof(uint64_t) * B->dv_words()));
  return GG_OK;
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

  // the quantum's steps, tail, RCCL, commit + import and the words' copy, one
  // sync per attempt; a failure (a wrong stream included) turns into the
  // error flag of the round, which every rank still takes part in
  const bool wrong_stream = s != ctx->last_stream;        // the context's kernels run on last_stream
  uint64_t* dv_own = B->dv;
  uint64_t* dv_all = B->dv + kRoundWords;
  uint64_t* counts = B->dv + (size_t)(1 + W) * kRoundWords;
  const uint64_t* h = B->host;
  uint32_t k0 = 0;
  for (int attempt = 0;; ++attempt) {
    uint32_t herr = 0;
    std::string emsg;
    gg_status est = GG_OK;
    if (wrong_stream) est = gg_fail(GG_ERR_INVALID, "gg_round_exchange needs the stream of gg_coherent_begin");
    // the batch: the largest of the last four quanta's steps + 3, doubling on a
    // repeat.  A step past the quantum's end costs three empty launches (~8
    // µs), a short batch a whole repeated round (~40 µs): margins 0 / 1 / 2 / 3
    // measured 62 / 44 / 45 / 35 µs per quantum (bench exchange, one rank)
    uint32_t nb = 0;
    for (uint32_t x : B->steps_hist) nb = std::max(nb, x);
    nb = std::min<uint32_t>(256, (nb + kBatchMargin) << std::min(attempt, 4));
    if (!est) est = gg_coh_steps_async(ctx, q, k0, nb);
    if (est) { herr = GG_DERR_STATE; emsg = gg_last_error(); }
    if (gg_status st = gg_coh_round_tail(ctx, B->send, (uint32_t)W, per, region, herr, dv_own)) return st;
    if (wrong_stream) GG_HIP(hipStreamSynchronize(ctx->last_stream));   // the slots and words before RCCL reads them on s
    if (W > 1) {                                           // the peers' slots (the own one is imported in place)
      GG_NCCL(ncclGroupStart());
      for (int r = 0; r < W; ++r) {
        if (r == R) continue;
        GG_NCCL(ncclSend(B->send + (size_t)r * (region + 1), sbytes, ncclUint8, r, comm, s));
        GG_NCCL(ncclRecv(B->recv + (size_t)r * (region + 1), sbytes, ncclUint8, r, comm, s));
      }
      GG_NCCL(ncclGroupEnd());
    }
    GG_NCCL(ncclAllGather(dv_own, dv_all, kRoundWords, ncclUint64, comm, s));
    if (wrong_stream) {                                    // this rank failed: nothing to import
      GG_HIP(hipStreamSynchronize(s));
      return gg_fail(est, "%s", emsg.c_str());
    }
    if (gg_status st = gg_coh_round_import(ctx, q, B->send, B->recv, (uint32_t)W, (uint32_t)R, region, slot, dv_all, counts))
      return st;
    GG_HIP(hipMemcpyAsync(B->host, dv_all, sizeof(uint64_t) * ((size_t)W * kRoundWords + 2 * (size_t)W),
                          hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    gg_coh_harvest(ctx);
    uint64_t err = 0, notdone = 0;
    for (int r = 0; r < W; ++r) { err |= h[r * kRoundWords + 3]; notdone |= h[r * kRoundWords + 6]; }
    if (err) {
      if (herr) return gg_fail(est ? est : GG_ERR_STATE, "%s", emsg.c_str());
      if (gg_status st = gg_coh_check(ctx)) return st;
      return gg_fail(GG_ERR_STATE, "quantum %llu failed on another rank", (unsigned long long)q);
    }
    if (notdone) { k0 += nb; continue; }                  // some rank's quantum is still running
    break;
  }
  // the reduced words: sent, active, blocked (sums), largest slot count (max),
  // least next start (min), the quantum's steps on this rank
  uint64_t msgs = 0, active = 0, blocked = 0, mx = 0, mn = ~0ull;
  for (int r = 0; r < W; ++r) {
    const uint64_t* w = h + (size_t)r * kRoundWords;
    msgs += w[0]; active += w[1]; blocked += w[2]; mx = std::max(mx, w[4]); mn = std::min(mn, w[5]);
  }
  B->steps_hist[B->hist_i++ & 3] = (uint32_t)std::max<uint64_t>(1, h[(size_t)R * kRoundWords + 7]);
  // a slot overflowed somewhere: every rank takes the sized round (the counts are known on both sides now)
  if (mx > slot) {
    const uint64_t* sc = h + (size_t)W * kRoundWords;
    const uint64_t* rc = sc + W;
    {                                                      // the own slot's tail: a local copy into the receive slot
      const size_t o = (size_t)R * (region + 1);
      GG_HIP(hipMemcpyAsync(B->recv + o, B->send + o, sizeof(gg_cmsg) * (1 + std::max(sc[R], slot)),
                            hipMemcpyDeviceToDevice, s));
    }
    if (W > 1) {
      GG_NCCL(ncclGroupStart());
      for (int r = 0; r < W; ++r) {
        if (r == R) continue;
        const size_t o = (size_t)r * (region + 1) + 1 + slot;
        if (sc[r] > slot) GG_NCCL(ncclSend(B->send + o, sizeof(gg_cmsg) * (sc[r] - slot), ncclUint8, r, comm, s));
        if (rc[r] > slot) GG_NCCL(ncclRecv(B->recv + o, sizeof(gg_cmsg) * (rc[r] - slot), ncclUint8, r, comm, s));
      }
      GG_NCCL(ncclGroupEnd());
    }
    if (gg_status st = gg_coh_import_slots(ctx, B->recv, (uint32_t)W, region, slot, region, false, nullptr)) return st;
    GG_HIP(hipStreamSynchronize(s));
  }
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
