// gg_core.hip — core timing of trace-driven tiles.
//
// SimpleCoreModel::handleInstruction (common/tile/core/models/
// simple_core_model.cc:43-96) over the per-access results of a coherent run:
// an access (a record without GG_META_CONT and the CONT line records after
// it) is one instruction whose static cost is its gap cycles
// (execution_unit_stall_time += cost, :86) with one memory operand whose
// latency is the sum of its line latencies (Core::initiateMemoryAccess's
// final - initial time, core.cc:239-256; read operands :62-72, write
// operands :73-83); curr_time += memory stall + cost (:88);
// CoreModel::updatePipelineStallCounters (core_model.cc:260-264) sums both.
//
// The model is a per-tile sum over the trace, so the device pass is a
// segmented reduction streamed from HBM: 12 algorithmic bytes per record
// (4-B meta word + 8-B access word; addresses are not read).  Tasks of up to
// kTaskRecords records of one tile, one wave each, 4 x 64 records in flight
// per iteration; a CONT record takes the WRITE bit of the access it belongs
// to from the last head before it (ballot over the wave, carried across
// iterations, looked up behind the task's first record; a CONT record at the
// tile's start or right after a BARRIER is a head, as in the oracle).  A BARRIER record
// with a stall is the SyncInstruction of sync_client.cc:306-314 (dynamic:
// curr_time += stall, CoreModel::updateDynamicInstructionCounters,
// core_model.cc:237-250).
#include "gg_internal.h"

namespace {

constexpr uint32_t kCoreWaves = 4;                 // waves per workgroup
constexpr uint64_t kTaskRecords = 16384;           // records per task (one wave)

struct CoreTask { uint64_t begin, end, tile_begin; uint32_t tile, pad; };

__device__ __forceinline__ uint32_t rec_write(uint32_t m) { return m & GG_META_WRITE; }

__global__ void __launch_bounds__(64 * kCoreWaves) k_core_model(const uint32_t* __restrict__ meta,
                                                                const uint64_t* __restrict__ acc,
                                                                const CoreTask* __restrict__ tasks, uint32_t ntasks,
                                                                uint64_t gap_ps, uint64_t* stats)
{
  const uint32_t w = blockIdx.x * kCoreWaves + (threadIdx.x >> 6), ln = threadIdx.x & 63;
  if (w >= ntasks) return;
  const CoreTask tk = tasks[w];
  // the access the task's first record belongs to: its head is the last
  // non-CONT record at or before it (CONT records follow their head)
  // (a CONT record right after a BARRIER or at the tile's start has no head
  // before it: it is a head itself, as in the oracle's scan)
  uint64_t j = tk.begin;
  while (j > tk.tile_begin && (meta[j] & GG_META_CONT) && meta[j] != GG_META_BARRIER && meta[j - 1] != GG_META_BARRIER) --j;
  uint32_t carry = rec_write(meta[j]);
  uint32_t prevm = tk.begin > tk.tile_begin ? meta[tk.begin - 1] : GG_META_BARRIER;   // the record before lane 0's
  uint64_t n_ins = 0, ex = 0, rd = 0, wr = 0, ns = 0, sy = 0;
  const uint64_t below = ln == 63 ? ~0ull : ((2ull << ln) - 1);   // lanes <= ln
  for (uint64_t b = tk.begin; b < tk.end; b += 256) {
    uint32_t m[4];
    uint64_t a[4];
    bool vl[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t r = b + 64 * u + ln;
      vl[u] = r < tk.end;
      m[u] = vl[u] ? meta[r] : GG_META_CONT;
      a[u] = vl[u] ? acc[r] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool bar = m[u] == GG_META_BARRIER;            // a released barrier: the SyncInstruction
      const uint32_t up = (uint32_t)__shfl((int)m[u], (int)((ln + 63) & 63));
      const uint32_t pm = ln == 0 ? prevm : up;            // the previous record's meta
      prevm = (uint32_t)__shfl((int)m[u], 63);
      const bool head = vl[u] && (!(m[u] & GG_META_CONT) || pm == GG_META_BARRIER);   // (no padding lane)
      const uint64_t heads = __ballot(head);
      const uint64_t mine = heads & below;
      const uint32_t own = rec_write(m[u]);
      const uint32_t hl = mine ? 63u - (uint32_t)__builtin_clzll(mine) : ln;
      const uint32_t from = __shfl(own, (int)hl);
      const uint32_t op = mine ? from : carry;
      if (heads) carry = __shfl(own, 63 - __builtin_clzll(heads));
      const uint64_t lat = a[u] >> 2;
      if (bar) { if (lat) { ++n_ins; ++ns; sy += lat; } continue; }
      if (head) { ++n_ins; ex += (uint64_t)((m[u] & 0x7FFFFFFFu) >> 1) * gap_ps; }
      if (op) wr += lat; else rd += lat;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n_ins += __shfl_xor(n_ins, o); ex += __shfl_xor(ex, o);
    rd += __shfl_xor(rd, o); wr += __shfl_xor(wr, o);
    ns += __shfl_xor(ns, o); sy += __shfl_xor(sy, o);
  }
  if (ln == 0) {
    unsigned long long* s = (unsigned long long*)(stats + (size_t)tk.tile * GG_NUM_CORE_STATS);
    atomicAdd(s + GG_CORE_INSTRUCTIONS, (unsigned long long)n_ins);
    atomicAdd(s + GG_CORE_TIME_PS, (unsigned long long)(ex + rd + wr + sy));
    atomicAdd(s + GG_CORE_SYNC_INSTRUCTIONS, (unsigned long long)ns);
    atomicAdd(s + GG_CORE_SYNC_STALL_PS, (unsigned long long)sy);
    atomicAdd(s + GG_CORE_MEMORY_STALL_PS, (unsigned long long)(rd + wr));
    atomicAdd(s + GG_CORE_EXECUTION_STALL_PS, (unsigned long long)ex);
    atomicAdd(s + GG_CORE_L1D_READ_STALL_PS, (unsigned long long)rd);
    atomicAdd(s + GG_CORE_L1D_WRITE_STALL_PS, (unsigned long long)wr);
  }
}

uint64_t cycle_ps(double f_ghz) { return (uint64_t)ceil(((double)1000 * 1) / f_ghz); }   // Latency(1, f).toPicosec

}  // namespace

void gg_core_free(gg_ctx* ctx)
{
  if (ctx->core_dev) hipFree(ctx->core_dev);
  if (ctx->core_tasks) hipFree(ctx->core_tasks);
  ctx->core_dev = nullptr; ctx->core_tasks = nullptr; ctx->core_task_cap = 0; ctx->core_valid = false;
}

extern "C" {

gg_status gg_core_model_run(gg_ctx* ctx, const gg_trace* tr, const uint64_t* access_out_dev, void* stream)
{
  if (!ctx || !tr || !tr->tile_offsets) return gg_fail(GG_ERR_INVALID, "gg_core_model_run: NULL argument");
  const uint32_t T = ctx->cfg.num_tiles;
  const uint64_t* off = tr->tile_offsets;
  if (off[0] != 0) return gg_fail(GG_ERR_INVALID, "gg_core_model_run: tile_offsets[0] != 0");
  for (uint32_t t = 0; t < T; ++t)
    if (off[t + 1] < off[t]) return gg_fail(GG_ERR_INVALID, "gg_core_model_run: tile offsets decrease");
  if (off[T] != tr->num_records) return gg_fail(GG_ERR_INVALID, "gg_core_model_run: tile_offsets[T] != num_records");
  if (tr->num_records && (!tr->meta_dev || !access_out_dev))
    return gg_fail(GG_ERR_INVALID, "gg_core_model_run: NULL meta or access words");
  if (!(ctx->cfg.frequency_ghz > 0)) return gg_fail(GG_ERR_INVALID, "gg_core_model_run: frequency %g", ctx->cfg.frequency_ghz);
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  std::vector<CoreTask> tasks;
  for (uint32_t t = 0; t < T; ++t)
    for (uint64_t b = off[t]; b < off[t + 1]; b += kTaskRecords)
      tasks.push_back(CoreTask{b, std::min(off[t + 1], b + kTaskRecords), off[t], t, 0});
  if (tasks.size() > 0xFFFFFFFFull / 2) return gg_fail(GG_ERR_RANGE, "gg_core_model_run: trace too long");
  if (!ctx->core_dev) GG_HIP(hipMalloc((void**)&ctx->core_dev, sizeof(uint64_t) * T * GG_NUM_CORE_STATS));
  if (tasks.size() > ctx->core_task_cap) {
    if (ctx->core_tasks) hipFree(ctx->core_tasks);
    ctx->core_tasks = nullptr; ctx->core_task_cap = 0;
    GG_HIP(hipMalloc(&ctx->core_tasks, sizeof(CoreTask) * tasks.size()));
    ctx->core_task_cap = tasks.size();
  }
  GG_HIP(hipMemsetAsync(ctx->core_dev, 0, sizeof(uint64_t) * T * GG_NUM_CORE_STATS, s));
  if (!tasks.empty()) {
    GG_HIP(hipMemcpyAsync(ctx->core_tasks, tasks.data(), sizeof(CoreTask) * tasks.size(), hipMemcpyHostToDevice, s));
    const uint32_t nt = (uint32_t)tasks.size();
    gg_timer_begin(ctx, "core_model", s);
    hipLaunchKernelGGL(k_core_model, dim3((nt + kCoreWaves - 1) / kCoreWaves), dim3(64 * kCoreWaves), 0, s,
                       tr->meta_dev, access_out_dev, (const CoreTask*)ctx->core_tasks, nt,
                       cycle_ps(ctx->cfg.frequency_ghz), ctx->core_dev);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "core_model", s);
  }
  ctx->core_valid = true;
  return GG_OK;
}

gg_status gg_core_get_stats(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "gg_core_get_stats: NULL argument");
  if (!ctx->core_valid) return gg_fail(GG_ERR_STATE, "gg_core_get_stats: gg_core_model_run has not run");
  hipSetDevice(ctx->device);
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  GG_HIP(hipMemcpy(out, ctx->core_dev, sizeof(uint64_t) * ctx->cfg.num_tiles * GG_NUM_CORE_STATS,
                   hipMemcpyDeviceToHost));
  return GG_OK;
}

}  // extern "C"
