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
// left blocked inside RCCL.  A failure found after a round's collective (the
// commit / import of unpack, the sized import of finish) cannot reach the
// words its peers already hold: it is kept as the rank's pending failure, the
// rank decides this round like its peers, and its next pack turns it into the
// error flag of its words — every rank returns it from that round's unpack.
// Only when this round ends the run (no peer will post another round) does
// the rank return the pending failure alone.
#include "gg_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kBatchMargin = 3;      // steps launched past the recent quanta's largest (see the round)
constexpr uint64_t kSlotDefault = 1024;   // records per peer and quantum sent in the fixed round (64 KB)
static_assert(GG_ROUND_WORDS == kRoundWords, "gg_internal.h kRoundWords");

struct RoundBufs {
  gg_cmsg* send = nullptr; gg_cmsg* recv = nullptr;   // [world][1 + region] each
  uint64_t* dv = nullptr;                             // [1 + world][kRoundWords] own, gathered; [2 * world] slot counts
  uint64_t* host = nullptr;                           // pinned copy of the gathered words and counts
  uint64_t region = 0; int world = 0;
  uint32_t steps_hist[4] = {8, 8, 8, 8};              // steps of the last quanta (the batch predictor)
  uint32_t hist_i = 0;
  // the round in progress (pack .. unpack / finish)
  uint32_t rank = 0, per = 0, k0 = 0, nb = 0, attempt = 0;
  uint64_t q = 0, slot = 0;
  bool again = false;                                 // unpack said GG_ROUND_AGAIN: the next pack continues q
  uint32_t herr = 0;                                  // this rank's local failure (its error flag in the words)
  gg_status est = GG_OK;
  std::string emsg;
  gg_status pend = GG_OK;                             // a failure after the collective: the next round's flag
  std::string pmsg;
  uint64_t gen = 0;                                   // the coherent run (gg_coh_generation) the round belongs to
  uint32_t nunpack = 0, nfinish = 0;                  // unpack / finish calls of this run (test knobs)
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

gg_status bufs_for(gg_ctx* ctx, RoundBufs*& B, int world, uint32_t rank, uint64_t region)
{
  B = static_cast<RoundBufs*>(gg_round_state(ctx));
  if (B && B->world == world && B->region >= region) return GG_OK;
  if (B) bufs_free(B);
  gg_round_state_set(ctx, nullptr, nullptr);
  B = new RoundBufs();
  B->region = region; B->world = world; B->rank = rank;
  gg_round_state_set(ctx, B, bufs_free);
  const size_t slots = (size_t)world * (region + 1);
  GG_HIP(hipMalloc((void**)&B->send, sizeof(gg_cmsg) * slots));
  GG_HIP(hipMalloc((void**)&B->recv, sizeof(gg_cmsg) * slots));
  GG_HIP(hipMalloc((void**)&B->dv, sizeof(uint64_t) * B->dv_words()));
  GG_HIP(hipHostMalloc((void**)&B->host, sizeof(uint64_t) * B->dv_words()));
  // test knob: the first batches' step counts per rank ("n0,n1,...", rank r
  // takes entry r mod the list): a short first batch on one rank makes the
  // round repeat while the other ranks have finished the quantum
  if (const char* e = getenv("GG_ROUND_BATCH0")) {
    std::vector<uint32_t> v;
    for (const char* c = e; *c;) { v.push_back((uint32_t)strtoul(c, (char**)&c, 10)); if (*c == ',') ++c; else break; }
    if (!v.empty()) for (uint32_t& x : B->steps_hist) x = std::max<uint32_t>(1, v[(size_t)B->rank % v.size()]);
  }
  return GG_OK;
}

uint64_t slot_records(uint64_t region)
{
  const char* e = getenv("GG_ROUND_SLOT");          // test knob: a small slot forces the overflow round
  uint64_t v = e ? strtoull(e, nullptr, 10) : kSlotDefault;
  return std::max<uint64_t>(1, std::min(v, region));
}

RoundBufs* bufs_of(gg_ctx* ctx) { return static_cast<RoundBufs*>(gg_round_state(ctx)); }

// test knob: GG_ROUND_FAIL_IMPORT / GG_ROUND_FAIL_FINISH = "rank,n" makes the
// n-th (0-based) unpack / finish of this run on that rank fail after the
// collective, as a failed commit or import would
bool knob_fail(const char* name, uint32_t rank, uint32_t n)
{
  const char* e = getenv(name);
  if (!e || !*e) return false;
  char* c = nullptr;
  const unsigned long r = strtoul(e, &c, 10);
  if (!c || *c != ',') return false;
  return r == rank && strtoul(c + 1, nullptr, 10) == n;
}

// a local failure after the collective: kept for the next round (the first one wins)
void set_pending(RoundBufs* B, gg_status st, const std::string& msg)
{
  if (B->pend) return;
  B->pend = st ? st : GG_ERR_STATE;
  B->pmsg = msg;
}

void fill_io(const RoundBufs* B, gg_round_io* io)
{
  io->send = B->send; io->recv = B->recv;
  io->words_own = B->dv; io->words_all = B->dv + kRoundWords;
  io->stride = B->region + 1; io->slot = B->slot;
  io->send_count = B->host + (size_t)B->world * kRoundWords;
  io->recv_count = io->send_count + B->world;
}

// pack with an extra local failure (gg_round_exchange's wrong stream)
gg_status round_pack(gg_ctx* ctx, uint32_t W, uint32_t R, uint64_t q, gg_round_io* io, gg_status xerr, const char* xmsg)
{
  if (!ctx || !io) return gg_fail(GG_ERR_INVALID, "NULL argument");
  const gg_config& c = ctx->cfg;
  const uint32_t K = c.num_shards ? c.num_shards : 1;
  if (W == 0 || R >= W) return gg_fail(GG_ERR_INVALID, "rank %u of %u ranks", R, W);
  if (K % W) return gg_fail(GG_ERR_INVALID, "%u logical shards do not split over %u ranks", K, W);
  const uint32_t per = K / W;
  const uint32_t k1 = c.shard_end ? c.shard_end : K;
  if (c.shard_begin != R * per || k1 != (R + 1) * per)
    return gg_fail(GG_ERR_INVALID, "rank %u must own shards [%u, %u), the context owns [%u, %u)", R, R * per,
                   (R + 1) * per, c.shard_begin, k1);
  hipSetDevice(ctx->device);
  // These checks and the first round's buffers fail before anything is
  // enqueued: they depend only on arguments and on gg_coherent_begin having
  // run, which every rank of one program gets identically (the send buffer
  // of the first round is the one rank-local failure that cannot become the
  // round's error flag: there is no buffer).
  const uint64_t region = gg_coherent_msg_cap(ctx);
  if (!region) return gg_fail(GG_ERR_INVALID, "gg_coherent_begin first");
  RoundBufs* B = nullptr;
  if (gg_status st = bufs_for(ctx, B, (int)W, R, region)) return st;
  B->rank = R; B->per = per;
  const uint64_t gen = gg_coh_generation(ctx);
  if (B->gen != gen) {
    // a new run (gg_coherent_begin): nothing of an abandoned round carries over
    B->gen = gen; B->again = false; B->pend = GG_OK; B->pmsg.clear(); B->nunpack = 0; B->nfinish = 0;
  }
  if (B->again && B->q == q) { B->k0 += B->nb; ++B->attempt; }
  else { B->k0 = 0; B->attempt = 0; B->herr = 0; B->est = GG_OK; B->emsg.clear(); }
  B->again = false; B->q = q;
  if (B->pend) {                                       // the last round's failure becomes this round's flag
    if (!B->herr) { B->herr = GG_DERR_STATE; B->est = B->pend; B->emsg = B->pmsg; }
    B->pend = GG_OK; B->pmsg.clear();
  }
  B->slot = slot_records(region);
  // the batch: the largest of the last four quanta's steps + 3, doubling on a
  // repeat.  A step past the quantum's end costs three empty launches (~8
  // µs), a short batch a whole repeated round (~40 µs): margins 0 / 1 / 2 / 3
  // measured 62 / 44 / 45 / 35 µs per quantum (bench exchange, one rank)
  uint32_t nb = 0;
  for (uint32_t x : B->steps_hist) nb = std::max(nb, x);
  B->nb = std::min<uint32_t>(256, (nb + kBatchMargin) << std::min<uint32_t>(B->attempt, 4));
  if (xerr && !B->herr) { B->herr = GG_DERR_STATE; B->est = gg_fail(xerr, "%s", xmsg); B->emsg = gg_last_error(); }
  if (!B->herr) {
    if (gg_status st = gg_coh_steps_async(ctx, q, B->k0, B->nb)) { B->herr = GG_DERR_STATE; B->est = st; B->emsg = gg_last_error(); }
  }
  if (gg_status st = gg_coh_round_tail(ctx, B->send, W, per, region, B->herr, B->dv)) {
    // the tail did not run: the words say so (best effort), the transport still runs
    if (!B->herr) { B->herr = GG_DERR_STATE; B->est = st; B->emsg = gg_last_error(); }
    std::vector<uint64_t> w(kRoundWords, 0);
    w[3] = GG_DERR_STATE;
    hipMemcpyAsync(B->dv, w.data(), sizeof(uint64_t) * kRoundWords, hipMemcpyHostToDevice, ctx->last_stream);
    for (uint32_t r = 0; r < W; ++r)
      hipMemsetAsync(B->send + (size_t)r * (region + 1), 0, sizeof(gg_cmsg), ctx->last_stream);
  }
  fill_io(B, io);
  io->state = GG_ROUND_AGAIN;
  return GG_OK;
}

// the quantum's end after every slot is in: the reduced words decide
gg_status round_decide(gg_ctx* ctx, RoundBufs* B, gg_round_io* io)
{
  const uint64_t* h = B->host;
  const int W = B->world;
  uint64_t msgs = 0, active = 0, blocked = 0, mn = ~0ull;
  for (int r = 0; r < W; ++r) {
    const uint64_t* w = h + (size_t)r * kRoundWords;
    msgs += w[0]; active += w[1]; blocked += w[2]; mn = std::min(mn, w[5]);
  }
  const uint64_t q = B->q;
  const uint64_t qps = (uint64_t)ctx->cfg.quantum_ns * 1000ull;
  io->state = GG_ROUND_DONE;
  io->done = 0;
  if (active == 0 && msgs == 0) {
    io->done = 1; io->next_q = q;
    // the run ends here on every rank: a pending failure has no next round
    if (B->pend) { const gg_status p = B->pend; B->pend = GG_OK; return gg_fail(p, "%s", B->pmsg.c_str()); }
    return gg_coh_check(ctx);
  }
  if (msgs == 0 && blocked != 0) return gg_fail(GG_ERR_STATE, "coherent run deadlocked: tiles blocked with no message in flight");
  io->next_q = (msgs == 0) ? std::max<uint64_t>(q + 1, mn / qps) : q + 1;
  return GG_OK;
}

}  // namespace

gg_status gg_round_pack(gg_ctx* ctx, uint32_t world, uint32_t rank, uint64_t q, gg_round_io* io)
{
  return round_pack(ctx, world, rank, q, io, GG_OK, "");
}

gg_status gg_round_unpack(gg_ctx* ctx, gg_round_io* io)
{
  if (!ctx || !io) return gg_fail(GG_ERR_INVALID, "NULL argument");
  RoundBufs* B = bufs_of(ctx);
  if (!B || !ctx->coh) return gg_fail(GG_ERR_INVALID, "gg_round_pack first");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  const int W = B->world;
  uint64_t* dv_all = B->dv + kRoundWords;
  uint64_t* counts = B->dv + (size_t)(1 + W) * kRoundWords;
  // commit + import (nothing unless every rank's words are clean), then the
  // words to the host; a local failure here still copies the words, so this
  // rank decides like the others and reports its own error on top
  gg_status lerr = gg_coh_round_import(ctx, B->q, B->send, B->recv, (uint32_t)W, B->rank, B->region, B->slot, dv_all, counts);
  std::string lmsg = lerr ? gg_last_error() : "";
  if (!lerr && knob_fail("GG_ROUND_FAIL_IMPORT", B->rank, B->nunpack)) {
    lerr = GG_ERR_STATE;
    lmsg = "commit / import failed on rank " + std::to_string(B->rank) + " (GG_ROUND_FAIL_IMPORT)";
  }
  ++B->nunpack;
  GG_HIP(hipMemcpyAsync(B->host, dv_all, sizeof(uint64_t) * ((size_t)W * kRoundWords + 2 * (size_t)W),
                        hipMemcpyDeviceToHost, s));
  GG_HIP(hipStreamSynchronize(s));
  gg_coh_harvest(ctx);
  fill_io(B, io);
  const uint64_t* h = B->host;
  uint64_t err = 0, notdone = 0, mx = 0;
  for (int r = 0; r < W; ++r) {
    err |= h[r * kRoundWords + 3]; notdone |= h[r * kRoundWords + 6]; mx = std::max(mx, h[r * kRoundWords + 4]);
  }
  if (err) {
    io->state = GG_ROUND_DONE;
    B->again = false; B->pend = GG_OK; B->pmsg.clear();
    if (B->herr) return gg_fail(B->est ? B->est : GG_ERR_STATE, "%s", B->emsg.c_str());
    if (gg_status st = gg_coh_check(ctx)) return st;
    return gg_fail(GG_ERR_STATE, "quantum %llu failed on another rank", (unsigned long long)B->q);
  }
  // a failure after the collective: this round is decided like the peers'
  // (they hold clean words), the next round carries it to every rank
  if (lerr) set_pending(B, lerr, lmsg);
  if (notdone) { B->again = true; io->state = GG_ROUND_AGAIN; return GG_OK; }   // some rank's quantum is still running
  B->steps_hist[B->hist_i++ & 3] = (uint32_t)std::max<uint64_t>(1, h[(size_t)B->rank * kRoundWords + 7]);
  if (mx > B->slot) {
    // a slot overflowed somewhere: every rank takes the sized round (the
    // counts are known on both sides now); the own slot's tail is a local copy
    const uint64_t* sc = h + (size_t)W * kRoundWords;
    const size_t o = (size_t)B->rank * (B->region + 1);
    GG_HIP(hipMemcpyAsync(B->recv + o, B->send + o, sizeof(gg_cmsg) * (1 + std::max(sc[B->rank], B->slot)),
                          hipMemcpyDeviceToDevice, s));
    io->state = GG_ROUND_OVERFLOW;
    return GG_OK;
  }
  return round_decide(ctx, B, io);
}

gg_status gg_round_finish(gg_ctx* ctx, gg_round_io* io)
{
  if (!ctx || !io) return gg_fail(GG_ERR_INVALID, "NULL argument");
  RoundBufs* B = bufs_of(ctx);
  if (!B || !ctx->coh) return gg_fail(GG_ERR_INVALID, "gg_round_pack first");
  hipSetDevice(ctx->device);
  // a failed import is this rank's alone (its peers decide from the same
  // words and go on): pending, as in unpack
  gg_status st = gg_coh_import_slots(ctx, B->recv, (uint32_t)B->world, B->region, B->slot, B->region, false, nullptr);
  std::string msg = st ? gg_last_error() : "";
  if (!st && knob_fail("GG_ROUND_FAIL_FINISH", B->rank, B->nfinish)) {
    st = GG_ERR_STATE;
    msg = "sized import failed on rank " + std::to_string(B->rank) + " (GG_ROUND_FAIL_FINISH)";
  }
  ++B->nfinish;
  if (st) set_pending(B, st, msg);
  if (hipError_t e = hipStreamSynchronize(ctx->last_stream))
    set_pending(B, GG_ERR_STATE, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  return round_decide(ctx, B, io);
}

gg_status gg_round_exchange(gg_ctx* ctx, void* nccl_comm, void* stream, uint64_t q, uint64_t* next_q, int* done)
{
  if (!ctx || !nccl_comm || !next_q || !done) return gg_fail(GG_ERR_INVALID, "NULL argument");
  ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
  int W = 0, R = 0;
  GG_NCCL(ncclCommCount(comm, &W));
  GG_NCCL(ncclCommUserRank(comm, &R));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // the context's kernels run on last_stream; RCCL on `stream`.  A different
  // stream is a local failure: it becomes the round's error flag, and the
  // transport is still posted so that no peer is left blocked inside RCCL
  const bool wrong_stream = s != ctx->last_stream;
  gg_round_io io{};
  for (;;) {
    if (gg_status st = round_pack(ctx, (uint32_t)W, (uint32_t)R, q, &io, wrong_stream ? GG_ERR_INVALID : GG_OK,
                                  "gg_round_exchange needs the stream of gg_coherent_begin"))
      return st;
    if (wrong_stream) GG_HIP(hipStreamSynchronize(ctx->last_stream));   // the slots and words before RCCL reads them on s
    const size_t sbytes = sizeof(gg_cmsg) * (io.slot + 1);
    if (W > 1) {                                           // the peers' slots (the own one is imported in place)
      GG_NCCL(ncclGroupStart());
      for (int r = 0; r < W; ++r) {
        if (r == R) continue;
        GG_NCCL(ncclSend(io.send + (size_t)r * io.stride, sbytes, ncclUint8, r, comm, s));
        GG_NCCL(ncclRecv(io.recv + (size_t)r * io.stride, sbytes, ncclUint8, r, comm, s));
      }
      GG_NCCL(ncclGroupEnd());
    }
    GG_NCCL(ncclAllGather(io.words_own, io.words_all, kRoundWords, ncclUint64, comm, s));
    if (wrong_stream) GG_HIP(hipStreamSynchronize(s));     // RCCL's writes before the unpack reads them on last_stream
    if (gg_status st = gg_round_unpack(ctx, &io)) return st;
    if (io.state == GG_ROUND_AGAIN) continue;
    break;
  }
  if (io.state == GG_ROUND_OVERFLOW) {
    const uint64_t* sc = io.send_count;
    const uint64_t* rc = io.recv_count;
    if (W > 1) {
      GG_NCCL(ncclGroupStart());
      for (int r = 0; r < W; ++r) {
        if (r == R) continue;
        const size_t o = (size_t)r * io.stride + 1 + io.slot;
        if (sc[r] > io.slot) GG_NCCL(ncclSend(io.send + o, sizeof(gg_cmsg) * (sc[r] - io.slot), ncclUint8, r, comm, s));
        if (rc[r] > io.slot) GG_NCCL(ncclRecv(io.recv + o, sizeof(gg_cmsg) * (rc[r] - io.slot), ncclUint8, r, comm, s));
      }
      GG_NCCL(ncclGroupEnd());
    }
    if (wrong_stream) GG_HIP(hipStreamSynchronize(s));
    if (gg_status st = gg_round_finish(ctx, &io)) return st;
  }
  *next_q = io.next_q;
  *done = io.done;
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
