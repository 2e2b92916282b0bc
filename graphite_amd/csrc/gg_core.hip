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
#include "gg_dev.h"

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

// ---- IOCOOMCoreModel (common/tile/core/models/iocoom_core_model.cc) ---------
// One wave per tile, every piece of the model's state in registers: the 512
// register scoreboard entries as 8 per lane (register r in lane r & 63, slot
// r >> 6) with their units as 2-bit fields, the load queue's and the store
// buffer's entries one per lane (<= 64 each).  The instructions' fields are
// wave-uniform (read lane by lane from a 64-instruction window loaded as one
// 16-B record per lane), so the whole model runs as scalar control with
// readlanes; the store buffer's address match (isAddressAvailable) is one
// ballot.  Instructions of one tile are strictly serial (curr_time and the
// scoreboard): the parallelism is across tiles.
constexpr uint32_t kIoWaves = 1;   // one-wave blocks: 1.4 % faster than 4, 2 puts two tiles on some SIMDs (-25 %)
enum : uint32_t { kUnitInvalid = 0, kUnitLoad = 1, kUnitExec = 3 };   // CoreUnit (iocoom_core_model.h:14-20)

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l)
{
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), (int)l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
}
// max of two wave-uniform u64: the subtract's borrow decides, all on the
// scalar unit (the compiler forms a u64 compare of SGPRs with a VALU compare
// through VCC, a VALU latency on the instruction's chain)
// The error checks as arithmetic on words: a bool or-ed across checks is
// kept as a lane mask and widened through a VALU select and a readfirstlane
__device__ __forceinline__ uint32_t is_barrier(uint32_t m) { return (uint32_t)(((uint64_t)m + 1u) >> 32); }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b)
{
  uint32_t rlo, rhi, t0, t1;
  asm("s_sub_u32 %2, %4, %6\n\t"
      "s_subb_u32 %3, %5, %7\n\t"
      "s_cselect_b32 %0, %6, %4\n\t"
      "s_cselect_b32 %1, %7, %5"
      : "=&s"(rlo), "=&s"(rhi), "=&s"(t0), "=&s"(t1)
      : "s"((uint32_t)a), "s"((uint32_t)(a >> 32)), "s"((uint32_t)b), "s"((uint32_t)(b >> 32))
      : "scc");
  return (uint64_t)rhi << 32 | rlo;
}
typedef uint64_t u64x8 __attribute__((ext_vector_type(8)));

// A scoreboard entry is the register's time with its unit in the top two
// bits (one indexed read gives both); times of 2^62 ps or more are flagged.
constexpr uint64_t kTimeMask = (1ull << 62) - 1;

struct IoCore {
  uint32_t ln;
  u64x8 sb;                       // _register_scoreboard + _register_dependency_list: register
                                  // ln + 64 s in slot s, unit << 62 | time (a vector value: a
                                  // uniform slot index reads it by indirect register
                                  // addressing, no memory)
  uint64_t lsb;                   // LoadQueue::_scoreboard[ln]
  uint64_t ssb, sad;              // StoreQueue::_scoreboard[ln], _addresses[ln]
  uint32_t ln_q, sn_q, lidx, sidx;
  uint64_t sq_lanes;               // the store buffer's lanes (< sn_q) as a wave mask
  uint64_t l_last, s_last;        // the entries at prev(lidx) / prev(sidx): the last ones written
                                  // (rings written in order), kept on the scalar unit
  bool spec, rfo;
  uint64_t one;

  __device__ __forceinline__ void reg_entry(uint32_t r, uint32_t& hi, uint32_t& lo) const
  {
    const uint64_t x = sb[r >> 6];
    hi = (uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), (int)(r & 63));
    lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)(r & 63));
  }
  __device__ __forceinline__ void reg_write(uint32_t r, uint64_t e)
  {
    const uint32_t s = r >> 6;
    const uint64_t old = sb[s];
    sb[s] = ln == (r & 63) ? e : old;
  }
  // the queues' ring indices wrap by a compare, not a modulo (a scalar
  // division is a long VALU sequence on the instruction's chain)
  __device__ __forceinline__ static uint32_t next_of(uint32_t i, uint32_t n) { return i + 1 == n ? 0u : i + 1; }
  // LoadQueue::execute (:182-208): the allocate time, *completion
  __device__ __forceinline__ uint64_t lq_execute(uint64_t schedule, uint64_t lat, uint64_t& completion)
  {
    const uint64_t allocate = umax64(rl64(lsb, lidx), schedule), lastd = l_last;
    uint64_t dealloc;
    if (spec) { completion = allocate + lat; dealloc = umax64(completion, lastd + one); }
    else { completion = umax64(lastd, schedule) + lat; dealloc = completion; }
    if (ln == lidx) lsb = dealloc;
    l_last = dealloc;
    lidx = next_of(lidx, ln_q);
    return allocate;
  }
  // executeLoad (:140-153) with StoreQueue::isAddressAvailable (:296-309)
  __device__ __forceinline__ uint64_t load(uint64_t schedule, uint64_t a, uint64_t latency, uint64_t& completion)
  {
    // (one ballot per compare: their masks combine on the scalar unit)
    if (__builtin_amdgcn_ballot_w64(sad == a) & __builtin_amdgcn_ballot_w64(ssb >= schedule) & sq_lanes) {
      completion = schedule + one;
      return schedule;
    }
    return lq_execute(schedule, latency + one, completion);
  }
  // executeStore (:155-165) + StoreQueue::execute (:250-284)
  __device__ __forceinline__ uint64_t store(uint64_t schedule, uint64_t a, uint64_t latency)
  {
    const uint64_t lat = latency + one;
    const uint64_t last_load = l_last;
    const uint64_t allocate = umax64(rl64(ssb, sidx), schedule);
    const uint64_t last_store = s_last;
    const uint64_t dealloc = rfo ? umax64(umax64(allocate + lat, last_store + one), last_load)
                                 : umax64(umax64(schedule, last_store), last_load) + lat;
    if (ln == sidx) { ssb = dealloc; sad = a; }
    s_last = dealloc;
    sidx = next_of(sidx, sn_q);
    return allocate;
  }
};

// The tile's access stream, 64 accesses per window (lane l holds access
// base + l); indices are 32-bit and relative to the tile's first access
// (gg_iocoom_run checks the per-tile counts), so the window tests are scalar
// compares
struct IoAcc {
  const uint64_t* __restrict__ addr;
  const uint32_t* __restrict__ meta;
  const uint64_t* __restrict__ lat;
  uint32_t n, ln, base = 0, m = 0;
  uint64_t a = 0, l = 0;
  // Per-lane tallies of the windows, summed over the wave at the end: the
  // windows tile [0, n) exactly (k advances by one per access) and a run
  // with k == n at its end consumed every access, a BARRIER by a
  // SyncInstruction and any other by a memory operand (else `bad`), so the
  // access-side statistics need no scalar work per instruction.
  uint64_t d_lat = 0, s_lat = 0;                  // data / SyncInstruction latency sums
  uint32_t d_cnt = 0, s_cnt = 0, s_zero = 0;      // data accesses, stalls != 0, stalls == 0
  __device__ __forceinline__ void load(uint32_t b)
  {
    base = b;
    const uint32_t i = b + ln;
    a = i < n ? addr[i] : 0; m = i < n ? meta[i] : 0; l = i < n ? lat[i] : 0;
    const bool bar = m == GG_META_BARRIER, in = i < n;
    d_lat += in && !bar ? l : 0; d_cnt += in && !bar ? 1u : 0u;
    s_lat += bar ? l : 0; s_cnt += bar && l ? 1u : 0u; s_zero += bar && !l ? 1u : 0u;
  }
  __device__ __forceinline__ void get(uint32_t k, uint64_t& A, uint32_t& M, uint64_t& L)
  {
    if (k - base >= 64) load(k);
    const uint32_t j = k - base;
    A = rl64(a, j); M = (uint32_t)__builtin_amdgcn_readlane((int)m, (int)j); L = rl64(l, j);
  }
};

// F1: the clock is 1 GHz, an instruction's cost is 1000 ps per cycle (the
// exact integer form of lat_to_ps, without its per-call test)
template <bool F1>
__global__ void __launch_bounds__(64 * kIoWaves) k_iocoom(const uint4* __restrict__ ins, const uint64_t* __restrict__ offs,
                                                          const uint64_t* __restrict__ addr,
                                                          const uint32_t* __restrict__ meta,
                                                          const uint64_t* __restrict__ lat, uint32_t T,
                                                          gg_iocoom_params p, double f, uint64_t* stats, uint32_t* err)
{
  // the tile index is wave-uniform: readfirstlane'd, so its offsets load into
  // SGPRs and every loop over its instructions is scalar control (from a
  // thread-derived index the compiler had built exec-masked loops whose
  // uniform state — curr, k, the counters — lived in VGPRs)
  const uint32_t t = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * kIoWaves + (threadIdx.x >> 6)));
  const uint32_t ln = threadIdx.x & 63;
  if (t >= T) return;
  IoCore c;
  c.ln = ln;
  c.sb = u64x8{0, 0, 0, 0, 0, 0, 0, 0};
  c.lsb = 0; c.ssb = 0; c.sad = ~0ull;                              // INVALID_ADDRESS (fixed_types.h:36)
  c.ln_q = p.num_load_queue_entries; c.sn_q = p.num_store_queue_entries; c.lidx = 0; c.sidx = 0;
  c.sq_lanes = __builtin_amdgcn_ballot_w64(ln < c.sn_q);
  c.l_last = 0; c.s_last = 0;
  c.spec = p.speculative_loads_enabled != 0; c.rfo = p.multiple_outstanding_RFOs_enabled != 0;
  c.one = gg::lat_to_ps(1, f);
  uint64_t st[GG_NUM_IOCOOM_STATS];
#pragma unroll
  for (int k = 0; k < GG_NUM_IOCOOM_STATS; ++k) st[k] = 0;
  const uint64_t i0 = offs[t], k0 = offs[T + 1 + t];
  const uint32_t ni = (uint32_t)(offs[t + 1] - i0), k1 = (uint32_t)(offs[T + 1 + t + 1] - k0);
  const uint4* __restrict__ tins = ins + i0;
  IoAcc acc;
  acc.addr = addr + k0; acc.meta = meta + k0; acc.lat = lat + k0; acc.n = k1; acc.ln = ln;
  acc.load(0);
  uint32_t k = 0;
  uint64_t curr = 0;
  uint32_t bad = 0;                 // (a word, not a bool: the compiler kept a bool in a VGPR)
  uint64_t sum_ready = 0, sum_re = 0, sum_rr = 0, sum_lqr = 0, sum_rmr = 0, sum_wor = 0, n_atomic = 0, n_fence = 0;
  for (uint32_t b = 0; b < ni && !bad; b += 64) {
    const uint4 w = b + ln < ni ? tins[b + ln] : make_uint4(0, 0, 0, 0);
    const uint32_t cnt = ni - b < 64 ? ni - b : 64u;
    // No early exit inside a window: a failed check sets `bad` and the
    // instruction runs on (register indices masked, accesses past the stream
    // read as zeros, stream indices never wrap), so the body is straight-line
    // scalar code; `bad` ends the walk at the window's end.  The operand
    // checks run over the window's 64 instructions at once, before the walk.
    {                                       // lane-parallel over the window: one instruction per lane
      const uint32_t ops = (w.x >> 16) & 0xFFu, regs = w.x >> 24;
      const bool real = b + ln < ni && !(regs & GG_INS_SYNC);
      // the fences (core_model.cc:221-235)
      n_atomic += __builtin_popcountll(__builtin_amdgcn_ballot_w64(real && (ops & GG_INS_ATOMIC)));
      n_fence += __builtin_popcountll(__builtin_amdgcn_ballot_w64(real && (ops >> GG_INS_FENCE_SHIFT)));
      // the operand checks: at most six register operands, each < 512
      const uint32_t no = (regs & 7u) + ((regs >> 3) & 7u);
      const bool badl = no > 6 || (no > 0 && (w.y & 0xFE00u)) || (no > 1 && (w.y >> 25)) || (no > 2 && (w.z & 0xFE00u)) ||
                        (no > 3 && (w.z >> 25)) || (no > 4 && (w.w & 0xFE00u)) || (no > 5 && (w.w >> 25));
      bad |= __builtin_amdgcn_ballot_w64(real && badl) ? 1u : 0u;
    }
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)w.x, (int)j);
      // the register operands as a queue: reads, then writes, 16 bits each
      uint64_t rq = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)w.z, (int)j) << 32 |
                    (uint32_t)__builtin_amdgcn_readlane((int)w.y, (int)j);
      uint32_t rq2 = (uint32_t)__builtin_amdgcn_readlane((int)w.w, (int)j);
      auto reg = [&]() {
        const uint32_t r = (uint32_t)rq & 0xFFFFu;
        rq = rq >> 16 | (uint64_t)rq2 << 48; rq2 >>= 16;
        return r;
      };
      auto next_access = [&](uint64_t& A, uint32_t& M, uint64_t& L) {
        acc.get(k++, A, M, L);        // past the stream: zeros, and k != k1 at the end (k < 2^32:
      };                              // at most 6 accesses per instruction, 2^28 instructions)
      const uint32_t ops = (w0 >> 16) & 0xFFu, regs = w0 >> 24;
      if (regs & GG_INS_SYNC) {                                       // dynamic (:74-79)
        uint64_t A, L; uint32_t M;
        next_access(A, M, L);
        bad |= is_barrier(M) ^ 1u;
        curr += L;                                                    // (its counts: the window tallies)
      } else {
        const uint64_t cost = F1 ? 1000ull * (w0 & 0xFFFFu) : gg::lat_to_ps(w0 & 0xFFFFu, f);   // getCost (:70)
        const uint64_t ready = curr;                                  // no L1-I (:78-87)
        const uint32_t nr = regs & 7u, nw = (regs >> 3) & 7u;
        // :100-125, as selects (no branch per operand).  An entry's unit is
        // LOAD (1) or EXECUTION (3) once written and INVALID (0) only with
        // time 0, which no maximum below can take: the top bit picks the
        // accumulator, and an INVALID entry's "time > ready" never holds.
        uint64_t rl = ready, re = ready;
        for (uint32_t i = 0; i < nr; ++i) {
          const uint32_t r = reg();
          uint32_t hi, lo;
          c.reg_entry(r & (GG_IOCOOM_NUM_REGISTERS - 1), hi, lo);
          uint32_t hs = hi;
          asm("" : "+s"(hs));               // (opaque copy: else the test is folded into a VALU i64 compare)
          const bool ex = (int32_t)hs < 0;
          const uint64_t mx = umax64((uint64_t)(hi & 0x3FFFFFFFu) << 32 | lo, ex ? re : rl);
          rl = ex ? rl : mx;
          re = ex ? mx : re;
        }
        const uint64_t rr = umax64(rl, re);                           // :128-129
        uint64_t lqr = rr, rmr = rr;                                  // :133-152
        for (uint32_t i = 0; i < (ops & 3u); ++i) {
          uint64_t A, L; uint32_t M;
          next_access(A, M, L);
          bad |= M & GG_META_WRITE;                                   // a write or a BARRIER (all ones)
          uint64_t comp;
          const uint64_t alloc = c.load(rr, A, L, comp);
          lqr = umax64(lqr, alloc); rmr = umax64(rmr, comp);
        }
        const uint64_t wor = rmr + cost;                              // :158-166
        const bool smov = (ops & GG_INS_SIMPLE_MOV_LOAD) != 0;
        const uint64_t went = wor | (uint64_t)(smov ? kUnitLoad : kUnitExec) << 62;
        bad |= (uint32_t)(wor >> 62);
        for (uint32_t i = 0; i < nw; ++i) {                           // :172-184
          const uint32_t r = reg();
          c.reg_write(r & (GG_IOCOOM_NUM_REGISTERS - 1), went);
        }
        uint64_t sqr = wor;                                           // :186-201
        const uint32_t nwm = (ops >> 2) & 3u;
        for (uint32_t i = 0; i < nwm; ++i) {
          uint64_t A, L; uint32_t M;
          next_access(A, M, L);
          bad |= ((M & GG_META_WRITE) ^ 1u) | is_barrier(M);
          sqr = umax64(sqr, c.store(wor, A, L));
        }
        // :209-252; the memory / execution stall totals (core_model.cc:260-264)
        // are the sums of these parts, formed once after the loop
        // (selects: a simple-mov load stops at lqr, a store-free one at rmr)
        const bool st_on = !smov && nwm;
        const uint64_t rmr_e = smov ? lqr : rmr, wor_e = st_on ? wor : rmr_e, sqr_e = st_on ? sqr : wor_e;
        // the six stall parts are differences of the chain ready <= re <=
        // rr <= lqr <= rmr_e <= wor_e <= sqr_e: sums of its links (mod 2^64,
        // exact for the differences), the last one from curr at the end
        sum_ready += ready; sum_re += re; sum_rr += rr; sum_lqr += lqr; sum_rmr += rmr_e; sum_wor += wor_e;
        curr = sqr_e;
      }
    }
  }
  if (k != k1) bad = 1;
  // :72 (a SyncInstruction of zero stall is no instruction), :74-79, the
  // data operands: the window tallies summed over the wave
  auto wsum = [](uint64_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
  };
  st[GG_IOCOOM_INSTRUCTIONS] = ni - wsum(acc.s_zero);
  st[GG_IOCOOM_SYNC_INSTRUCTIONS] = wsum(acc.s_cnt);
  st[GG_IOCOOM_SYNC_STALL_PS] = wsum(acc.s_lat);
  st[GG_IOCOOM_DATA_ACCESSES] = wsum(acc.d_cnt);
  st[GG_IOCOOM_DATA_LATENCY_PS] = wsum(acc.d_lat);
  const uint64_t sum_sqr = sum_ready + (curr - st[GG_IOCOOM_SYNC_STALL_PS]);   // curr = the links + the syncs' stalls
  st[GG_IOCOOM_INTER_EXEC_STALL_PS] = sum_re - sum_ready;                    // :209-252
  st[GG_IOCOOM_INTER_L1D_STALL_PS] = sum_rr - sum_re;
  st[GG_IOCOOM_LOAD_QUEUE_STALL_PS] = sum_lqr - sum_rr;
  st[GG_IOCOOM_INTRA_L1D_STALL_PS] = sum_rmr - sum_lqr;
  st[GG_IOCOOM_INTRA_EXEC_STALL_PS] = sum_wor - sum_rmr;
  st[GG_IOCOOM_STORE_QUEUE_STALL_PS] = sum_sqr - sum_wor;
  st[GG_IOCOOM_IMPLICIT_MFENCES] = n_atomic;
  st[GG_IOCOOM_EXPLICIT_FENCES] = n_fence;
  st[GG_IOCOOM_TIME_PS] = curr;
  st[GG_IOCOOM_MEMORY_STALL_PS] = st[GG_IOCOOM_INTER_L1D_STALL_PS] + st[GG_IOCOOM_LOAD_QUEUE_STALL_PS] +
                                  st[GG_IOCOOM_INTRA_L1D_STALL_PS] + st[GG_IOCOOM_STORE_QUEUE_STALL_PS];
  st[GG_IOCOOM_EXECUTION_STALL_PS] = st[GG_IOCOOM_INTER_EXEC_STALL_PS] + st[GG_IOCOOM_INTRA_EXEC_STALL_PS];
  if (bad) { if (ln == 0) atomicOr(err, 1u); return; }
  // lane s stores statistic s (one vector store)
  uint64_t v = 0;
#pragma unroll
  for (int s = 0; s < GG_NUM_IOCOOM_STATS; ++s) v = ln == (uint32_t)s ? st[s] : v;
  if (ln < GG_NUM_IOCOOM_STATS) stats[(size_t)t * GG_NUM_IOCOOM_STATS + ln] = v;
}

uint64_t cycle_ps(double f_ghz) { return (uint64_t)ceil(((double)1000 * 1) / f_ghz); }   // Latency(1, f).toPicosec

}  // namespace

void gg_core_free(gg_ctx* ctx)
{
  if (ctx->core_dev) hipFree(ctx->core_dev);
  if (ctx->core_tasks) hipFree(ctx->core_tasks);
  ctx->core_dev = nullptr; ctx->core_tasks = nullptr; ctx->core_task_cap = 0; ctx->core_valid = false;
  if (ctx->io_stats) hipFree(ctx->io_stats);
  if (ctx->io_offs) hipFree(ctx->io_offs);
  if (ctx->io_err) hipFree(ctx->io_err);
  ctx->io_stats = nullptr; ctx->io_offs = nullptr; ctx->io_err = nullptr; ctx->io_valid = false;
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

gg_status gg_iocoom_run(gg_ctx* ctx, const gg_iocoom_params* params, const gg_ins* ins_dev,
                        const uint64_t* ins_tile_offsets, const uint64_t* acc_addr_dev, const uint32_t* acc_meta_dev,
                        const uint64_t* acc_lat_dev, const uint64_t* acc_tile_offsets, void* stream)
{
  if (!ctx || !params || !ins_tile_offsets || !acc_tile_offsets)
    return gg_fail(GG_ERR_INVALID, "gg_iocoom_run: NULL argument");
  const gg_iocoom_params p = *params;
  if (p.num_load_queue_entries - 1u >= 64u || p.num_store_queue_entries - 1u >= 64u)
    return gg_fail(GG_ERR_UNSUPPORTED, "gg_iocoom_run: queue entries %u / %u (1..64)", p.num_load_queue_entries,
                   p.num_store_queue_entries);
  const uint32_t T = ctx->cfg.num_tiles;
  for (const uint64_t* o : {ins_tile_offsets, acc_tile_offsets})
    for (uint32_t t = 0; t < T; ++t)
      if (o[t + 1] < o[t]) return gg_fail(GG_ERR_INVALID, "gg_iocoom_run: tile offsets decrease");
      else if (o[t + 1] - o[t] > (o == ins_tile_offsets ? 1ull << 28 : 1ull << 31))   // 32-bit tile-relative indices
        return gg_fail(GG_ERR_RANGE, "gg_iocoom_run: tile %u has %llu %s (at most 2^%d)", t,
                       (unsigned long long)(o[t + 1] - o[t]), o == ins_tile_offsets ? "instructions" : "accesses",
                       o == ins_tile_offsets ? 28 : 31);
  if (ins_tile_offsets[T] > ins_tile_offsets[0] && !ins_dev) return gg_fail(GG_ERR_INVALID, "gg_iocoom_run: NULL instructions");
  if (acc_tile_offsets[T] > acc_tile_offsets[0] && (!acc_addr_dev || !acc_meta_dev || !acc_lat_dev))
    return gg_fail(GG_ERR_INVALID, "gg_iocoom_run: NULL access stream");
  if (!(ctx->cfg.frequency_ghz > 0)) return gg_fail(GG_ERR_INVALID, "gg_iocoom_run: frequency %g", ctx->cfg.frequency_ghz);
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  if (!ctx->io_stats) {
    GG_HIP(hipMalloc((void**)&ctx->io_stats, sizeof(uint64_t) * T * GG_NUM_IOCOOM_STATS));
    GG_HIP(hipMalloc((void**)&ctx->io_offs, sizeof(uint64_t) * 2 * (T + 1)));
    GG_HIP(hipMalloc((void**)&ctx->io_err, sizeof(uint32_t)));
  }
  std::vector<uint64_t> offs(2 * (size_t)(T + 1));
  std::copy(ins_tile_offsets, ins_tile_offsets + T + 1, offs.begin());
  std::copy(acc_tile_offsets, acc_tile_offsets + T + 1, offs.begin() + T + 1);
  GG_HIP(hipMemcpyAsync(ctx->io_offs, offs.data(), sizeof(uint64_t) * offs.size(), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemsetAsync(ctx->io_stats, 0, sizeof(uint64_t) * T * GG_NUM_IOCOOM_STATS, s));
  GG_HIP(hipMemsetAsync(ctx->io_err, 0, sizeof(uint32_t), s));
  if (T) {
    gg_timer_begin(ctx, "iocoom", s);
    hipLaunchKernelGGL(ctx->cfg.frequency_ghz == 1.0 ? k_iocoom<true> : k_iocoom<false>, dim3((T + kIoWaves - 1) / kIoWaves),
                       dim3(64 * kIoWaves), 0, s,
                       reinterpret_cast<const uint4*>(ins_dev), (const uint64_t*)ctx->io_offs, acc_addr_dev,
                       acc_meta_dev, acc_lat_dev, T, p, ctx->cfg.frequency_ghz, ctx->io_stats, ctx->io_err);
    GG_HIP(hipGetLastError());
    gg_timer_end(ctx, "iocoom", s);
  }
  ctx->io_valid = true;
  return GG_OK;
}

gg_status gg_iocoom_get_stats(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "gg_iocoom_get_stats: NULL argument");
  if (!ctx->io_valid) return gg_fail(GG_ERR_STATE, "gg_iocoom_get_stats: gg_iocoom_run has not run");
  hipSetDevice(ctx->device);
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  uint32_t e = 0;
  GG_HIP(hipMemcpy(&e, ctx->io_err, sizeof e, hipMemcpyDeviceToHost));
  if (e) return gg_fail(GG_ERR_STATE, "gg_iocoom_run: the instruction and access streams disagree, a register is out of range or a register time reached 2^62 ps");
  GG_HIP(hipMemcpy(out, ctx->io_stats, sizeof(uint64_t) * ctx->cfg.num_tiles * GG_NUM_IOCOOM_STATS,
                   hipMemcpyDeviceToHost));
  return GG_OK;
}

}  // extern "C"
