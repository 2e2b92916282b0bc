/*
 * gg_oracle.c — plain-C restatement of Graphite's memory-subsystem hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gg_oracle.h).  The shipped backend
 * (graphite_amd/) never links or calls this file; it is the checker for the
 * HIP kernels and the CPU baseline timed by bench.py.
 *
 * Citations are path:line in the reference (nmtrmail/Graphite).
 * Compile with -ffp-contract=off: the double/float arithmetic below must
 * round exactly like the reference's (time_types.h:81-109,
 * queue_model_m_g_1.cc:18-56).
 */
#include "gg_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================== */
/* misc/utils.cc:18-34                                                       */
/* ======================================================================== */
static int floor_log2(uint32_t n) { int p = -1; while (n) { n >>= 1; ++p; } return p; }
static int ceil_log2(uint32_t n) { int p = floor_log2(n); return ((1u << p) == n) ? p : p + 1; }

/* misc/time_types.h:81-109 */
static uint64_t lat_to_ps(uint64_t cycles, double f) { return (uint64_t)ceil(((double)1000 * cycles) / (double)f); }
static uint64_t time_to_cycles(uint64_t ps, double f) { return (uint64_t)ceil(((double)ps * (double)f) / (double)1.0e3); }

/* ======================================================================== */
/* Synthetic workloads        */
/* ======================================================================== */
static uint64_t mix64(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t i)
{
  return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
}

void oracle_gen_uniform(uint32_t tile, uint64_t first, uint64_t n, uint32_t lines_log2,
                        uint32_t base_shift, uint64_t* addr, uint32_t* meta)
{
  const uint64_t seed = 0x9E3779B97F4A7C15ull ^ (uint64_t)tile;
  const uint64_t mask = (1ull << lines_log2) - 1;
  for (uint64_t k = 0; k < n; ++k) {
    uint64_t z = oracle_splitmix64_at(seed, first + k);
    addr[k] = ((uint64_t)tile << base_shift) + ((z & mask) << 6);
    meta[k] = (((z >> 32) % 3) == 0) ? GG_META_WRITE : 0u;
  }
}

/* configs[2..4] hotspot generator: record i of tile t,
 * z = SplitMix64(0x9E3779B97F4A7C15 ^ t) step first+i+1;
 *   hot     iff ((z >> 40) & 0xFF) < hot_frac256  -> line (z & 0xFFFFFFFF) % hot_lines of the
 *                                                   shared region at 1 << 44
 *   private otherwise                            -> line z & (2^lines_log2 - 1) at t << base_shift
 *   WRITE   iff ((z >> 32) & 0xFF) % 3 == 0
 *   gap     = ctz(((z >> 48) & 0xFF) | 0x100) + ctz(((z >> 56) & 0xFF) | 0x100) cycles (mean ~2) */
void oracle_gen_hotspot(uint32_t tile, uint64_t first, uint64_t n, uint32_t lines_log2,
                        uint32_t base_shift, uint32_t hot_lines, uint32_t hot_frac256,
                        uint64_t* addr, uint32_t* meta)
{
  const uint64_t seed = 0x9E3779B97F4A7C15ull ^ (uint64_t)tile;
  const uint64_t mask = (1ull << lines_log2) - 1;
  for (uint64_t k = 0; k < n; ++k) {
    uint64_t z = oracle_splitmix64_at(seed, first + k);
    int hot = hot_lines && (((z >> 40) & 0xFF) < hot_frac256);
    if (hot) addr[k] = (1ull << 44) + ((z & 0xFFFFFFFFull) % hot_lines) * 64ull;
    else addr[k] = ((uint64_t)tile << base_shift) + ((z & mask) << 6);
    uint32_t gap = (uint32_t)__builtin_ctz((uint32_t)(((z >> 48) & 0xFF) | 0x100)) +
                   (uint32_t)__builtin_ctz((uint32_t)(((z >> 56) & 0xFF) | 0x100));
    meta[k] = ((((z >> 32) & 0xFF) % 3) == 0 ? GG_META_WRITE : 0u) | (gap << 1);
  }
}

/* configs[4] coherent stress generator: the recipe of gg_gen_stress_trace
 * (include/graphite_gpu.h).  Synthetic workload of the
 * SURVEY.md §8d config 5 description, not a reference algorithm.           */
static uint32_t stress_group(uint32_t t, uint32_t groups)
{
  uint32_t x = t + 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x % groups;
}
void oracle_gen_stress(uint32_t tile, uint64_t first, uint64_t n, uint32_t lines_log2, uint32_t base_shift,
                       uint32_t num_tiles, uint32_t pool_lines, uint32_t pool_frac256, uint64_t* addr, uint32_t* meta)
{
  const uint64_t seed = 0x9E3779B97F4A7C15ull ^ (uint64_t)tile;
  const uint64_t mask = (1ull << lines_log2) - 1;
  const uint32_t groups = num_tiles >= 128 ? num_tiles / 64 : 1;
  const uint32_t per_group = pool_lines / groups ? pool_lines / groups : 1;
  for (uint64_t k = 0; k < n; ++k) {
    uint64_t z = oracle_splitmix64_at(seed, first + k);
    int pool = pool_lines && (((z >> 40) & 0xFF) < pool_frac256);
    if (pool) addr[k] = (1ull << 45) + (uint64_t)(stress_group(tile, groups) + groups * ((uint32_t)(z & 0xFFFFFFFFull) % per_group)) * 64ull;
    else addr[k] = ((uint64_t)tile << base_shift) + ((z & mask) << 6);
    uint32_t gap = (uint32_t)__builtin_ctz((uint32_t)(((z >> 48) & 0xFF) | 0x100)) +
                   (uint32_t)__builtin_ctz((uint32_t)(((z >> 56) & 0xFF) | 0x100));
    meta[k] = (uint32_t)((z >> 32) & 1u) * GG_META_WRITE | (gap << 1);
  }
}

/* Core::initiateMemoryAccess line split (common/tile/core/core.cc:167-201) */
uint32_t oracle_split_lines(uint64_t addr, uint32_t size, uint32_t line, uint64_t* lines, uint32_t cap)
{
  if (size == 0) return 0;                          /* core.cc:145-155 */
  uint64_t begin = addr, end = addr + size;
  uint64_t ba = begin - (begin % line), ea = end - (end % line);
  uint32_t cnt = 0;
  for (uint64_t a = ba; a <= ea; a += line) {
    uint32_t off = (a == ba) ? (uint32_t)(begin % line) : 0;
    uint32_t sz;
    if (a == ea) { sz = (uint32_t)(end % line) - off; if (sz == 0) continue; }
    else sz = line - off;
    (void)sz;
    if (cnt < cap) lines[cnt] = a;
    ++cnt;
  }
  return cnt;
}

/* Multi-line accesses (core.cc:139-266) as line records: access i (byte addr,
 * size, meta) becomes lines first[i] .. first[i+1]-1; the first line keeps the
 * access's WRITE bit and gap, the others are GG_META_CONT (issued at the
 * previous line's completion, never cut at the lax barrier: one instruction).
 * A zero-size access makes no line (core.cc:145-155); its gap cycles move to
 * the tile's next access (the core clock keeps running).  Returns the number
 * of lines, or ~0 when a carried gap exceeds 30 bits.  line_addr / line_meta
 * may be NULL (count only).  tile_offsets: [tiles + 1] access offsets.      */
uint64_t oracle_split_accesses(const uint64_t* addr, const uint32_t* size, const uint32_t* meta,
                               const uint64_t* tile_offsets, uint32_t tiles, uint32_t line,
                               uint64_t* first, uint64_t* line_addr, uint32_t* line_meta)
{
  uint64_t nl = 0;
  uint64_t buf[64];
  for (uint32_t t = 0; t < tiles; ++t) {
    uint64_t carry = 0;
    for (uint64_t i = tile_offsets[t]; i < tile_offsets[t + 1]; ++i) {
      first[i] = nl;
      const uint64_t gap = carry + ((meta[i] & 0x7FFFFFFFu) >> 1);
      if (size[i] == 0) { carry = gap; continue; }
      carry = 0;
      if (gap >= (1ull << 30)) return ~0ull;
      /* an access spans at most size / line + 2 lines: count first, then fill */
      uint32_t k = oracle_split_lines(addr[i], size[i], line, buf, 64);
      for (uint32_t j = 0; j < k; ++j) {
        const uint64_t a = j < 64 ? buf[j] : (addr[i] - addr[i] % line) + (uint64_t)j * line;
        if (line_addr) line_addr[nl] = a;
        if (line_meta) line_meta[nl] = j == 0 ? (meta[i] & GG_META_WRITE) | ((uint32_t)gap << 1)
                                              : (meta[i] & GG_META_WRITE) | GG_META_CONT;
        ++nl;
      }
    }
  }
  if (tiles) first[tile_offsets[tiles]] = nl;
  return nl;
}

/* Per-access results of a split trace (core.cc:239-251): latency = the
 * access's final - initial time = the sum of its lines' latencies (each line
 * starts at the previous one's completion); misses = lines that did not hit
 * the L1-D on their first attempt (l1_cache_cntlr.cc:100-179).              */
void oracle_combine_accesses(const uint64_t* line_out, const uint64_t* first, uint64_t n,
                             uint64_t* latency_ps, uint32_t* misses)
{
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t lat = 0;
    uint32_t m = 0;
    for (uint64_t l = first[i]; l < first[i + 1]; ++l) {
      lat += line_out[l] >> 2;
      m += (line_out[l] & 3u) != GG_LVL_L1;
    }
    latency_ps[i] = lat;
    misses[i] = m;
  }
}

/* ======================================================================== */
/* Core timing: SimpleCoreModel (common/tile/core/models/simple_core_model.cc) */
/* ======================================================================== */
typedef struct {
  uint64_t instruction_count, curr_time;                     /* CoreModel (core_model.cc:31-45) */
  uint64_t total_sync_instructions, total_sync_instruction_stall_time;
  uint64_t total_memory_stall_time, total_execution_unit_stall_time;
  uint64_t total_l1icache_stall_time, total_l1dcache_read_stall_time, total_l1dcache_write_stall_time;
} o_core;

/* DynamicMemoryInfo {read, latency} of one access (core.cc:258-263) */
typedef struct { int read; uint64_t latency; } o_meminfo;

/* SimpleCoreModel::handleInstruction (simple_core_model.cc:43-96) for an
 * instruction of static cost `cost` with the memory operands `info` (one per
 * access in a trace).  No L1-I is modeled: modelICache contributes 0.       */
static void o_core_handle(o_core* c, uint64_t cost, const o_meminfo* info, int n)
{
  c->instruction_count++;                                            /* :50 */
  uint64_t memory_stall_time = 0, execution_unit_stall_time = 0;
  const uint64_t icache = 0;                                         /* :62-64 */
  memory_stall_time += icache;
  c->total_l1icache_stall_time += icache;
  for (int i = 0; i < n; ++i) {
    if (info[i].read) {                                              /* :69-78 */
      memory_stall_time += info[i].latency;
      c->total_l1dcache_read_stall_time += info[i].latency;
    } else {                                                         /* :79-88 */
      memory_stall_time += info[i].latency;
      c->total_l1dcache_write_stall_time += info[i].latency;
    }
  }
  execution_unit_stall_time += cost;                                 /* :90 */
  c->curr_time += memory_stall_time + execution_unit_stall_time;     /* :92 */
  c->total_memory_stall_time += memory_stall_time;                   /* core_model.cc:260-264 */
  c->total_execution_unit_stall_time += execution_unit_stall_time;
}

/* A tile's trace is its instruction stream: each access (a record without
 * GG_META_CONT and the CONT line records after it) is one instruction with
 * static cost = gap cycles (Latency(1, f) per cycle, the engine's gap rule)
 * and one memory operand, read unless the head record is a WRITE, whose
 * latency is Core::initiateMemoryAccess's final - initial time = the sum of
 * its line latencies (core.cc:239-256).                                    */
void oracle_core_model(const uint32_t* meta, const uint64_t* access_out, const uint64_t* tile_offsets,
                       uint32_t tiles, double frequency_ghz, uint64_t* stats)
{
  const uint64_t cyc = lat_to_ps(1, frequency_ghz);
  for (uint32_t t = 0; t < tiles; ++t) {
    o_core c;
    memset(&c, 0, sizeof c);
    uint64_t r = tile_offsets[t];
    const uint64_t e = tile_offsets[t + 1];
    while (r < e) {
      if (meta[r] == GG_META_BARRIER) {            /* SyncClient::barrierWait (sync_client.cc:306-314) */
        const uint64_t stall = access_out[r] >> 2;
        if (stall) {                               /* CoreModel::handleInstruction of a SyncInstruction */
          c.instruction_count++;                   /* (dynamic: core_model.cc:237-250) */
          c.curr_time += stall;
          c.total_sync_instructions++;
          c.total_sync_instruction_stall_time += stall;
        }
        ++r;
        continue;
      }
      o_meminfo info;
      info.read = !(meta[r] & GG_META_WRITE);
      info.latency = access_out[r] >> 2;
      const uint64_t cost = (uint64_t)((meta[r] & 0x7FFFFFFFu) >> 1) * cyc;
      for (++r; r < e && (meta[r] & GG_META_CONT) && meta[r] != GG_META_BARRIER; ++r) info.latency += access_out[r] >> 2;
      o_core_handle(&c, cost, &info, 1);
    }
    uint64_t* o = stats + (size_t)t * GG_NUM_CORE_STATS;
    memset(o, 0, sizeof(uint64_t) * GG_NUM_CORE_STATS);
    o[GG_CORE_INSTRUCTIONS] = c.instruction_count;
    o[GG_CORE_TIME_PS] = c.curr_time;
    o[GG_CORE_MEMORY_STALL_PS] = c.total_memory_stall_time;
    o[GG_CORE_EXECUTION_STALL_PS] = c.total_execution_unit_stall_time;
    o[GG_CORE_L1D_READ_STALL_PS] = c.total_l1dcache_read_stall_time;
    o[GG_CORE_L1D_WRITE_STALL_PS] = c.total_l1dcache_write_stall_time;
    o[GG_CORE_SYNC_INSTRUCTIONS] = c.total_sync_instructions;
    o[GG_CORE_SYNC_STALL_PS] = c.total_sync_instruction_stall_time;
  }
}

/* ======================================================================== */
/* Core timing: IOCOOMCoreModel (common/tile/core/models/iocoom_core_model.cc) */
/* ======================================================================== */
enum { IO_INVALID_UNIT = 0, IO_LOAD_UNIT = 1, IO_STORE_UNIT = 2, IO_EXECUTION_UNIT = 3 };   /* .h:14-20 */
#define IO_MAXQ 64
typedef struct {                     /* LoadQueue (:162-223) / StoreQueue (:225-322) */
  uint64_t sb[IO_MAXQ];              /* _scoreboard (deallocate times)           */
  uint64_t addr[IO_MAXQ];            /* _addresses (store queue)                 */
  uint32_t n, idx, flag;             /* _num_entries, _allocate_idx, speculative / multiple RFOs */
} o_ioq;
typedef struct {
  uint64_t sb[GG_IOCOOM_NUM_REGISTERS];      /* _register_scoreboard             */
  uint8_t dep[GG_IOCOOM_NUM_REGISTERS];      /* _register_dependency_list        */
  o_ioq lq, sq;
  uint64_t one;                              /* _ONE_CYCLE                        */
  uint64_t st[GG_NUM_IOCOOM_STATS];
} o_iocoom;

static inline uint64_t o_max(uint64_t a, uint64_t b) { return a > b ? a : b; }

/* LoadQueue::execute (:182-208): returns allocate time, *completion */
static uint64_t o_lq_execute(o_iocoom* c, uint64_t schedule, uint64_t lat, uint64_t* completion)
{
  o_ioq* q = &c->lq;
  const uint64_t allocate = o_max(q->sb[q->idx], schedule);
  const uint32_t last = (q->idx + q->n - 1) % q->n;
  uint64_t dealloc;
  if (q->flag) {                                   /* speculative loads */
    *completion = allocate + lat;
    dealloc = o_max(*completion, q->sb[last] + c->one);
  } else {
    *completion = o_max(q->sb[last], schedule) + lat;
    dealloc = *completion;
  }
  q->sb[q->idx] = dealloc;
  q->idx = (q->idx + 1) % q->n;
  return allocate;
}
/* StoreQueue::isAddressAvailable (:296-309): every entry, never-used ones included */
static int o_sq_available(const o_iocoom* c, uint64_t schedule, uint64_t a)
{
  for (uint32_t i = 0; i < c->sq.n; ++i)
    if (c->sq.addr[i] == a && c->sq.sb[i] >= schedule) return 1;
  return 0;
}
/* executeLoad (:140-153) */
static uint64_t o_io_load(o_iocoom* c, uint64_t schedule, uint64_t a, uint64_t latency, uint64_t* completion)
{
  const uint64_t lat = latency + c->one;
  if (o_sq_available(c, schedule, a)) { *completion = schedule + c->one; return schedule; }
  return o_lq_execute(c, schedule, lat, completion);
}
/* executeStore (:155-165) + StoreQueue::execute (:250-284) */
static uint64_t o_io_store(o_iocoom* c, uint64_t schedule, uint64_t a, uint64_t latency)
{
  const uint64_t lat = latency + c->one;
  const uint64_t last_load = c->lq.sb[(c->lq.idx + c->lq.n - 1) % c->lq.n];   /* getLastDeallocateTime */
  o_ioq* q = &c->sq;
  const uint64_t allocate = o_max(q->sb[q->idx], schedule);
  const uint32_t last = (q->idx + q->n - 1) % q->n;
  const uint64_t last_store = q->sb[last];
  uint64_t dealloc;
  if (q->flag) dealloc = o_max(o_max(allocate + lat, last_store + c->one), last_load);   /* multiple RFOs */
  else dealloc = o_max(o_max(schedule, last_store), last_load) + lat;
  q->sb[q->idx] = dealloc;
  q->addr[q->idx] = a;
  q->idx = (q->idx + 1) % q->n;
  return allocate;
}

/* IOCOOMCoreModel::handleInstruction (iocoom_core_model.cc:66-227) for one
 * gg_ins; its memory operands take the tile's next accesses (*k).  No L1-I:
 * modelICache contributes 0 (:78-81).  Returns 0, or -1 when the streams
 * disagree (the reference's LOG_ASSERT_ERRORs at :93-118,:129,:175).      */
static int o_io_handle(o_iocoom* c, uint64_t* curr, const gg_ins* in, const uint64_t* addr, const uint32_t* meta,
                       const uint64_t* lat, uint64_t* k, uint64_t kend, double f)
{
  uint64_t* st = c->st;
  st[GG_IOCOOM_INSTRUCTIONS]++;                                       /* :72 */
  if (in->regs & GG_INS_SYNC) {                                       /* dynamic (:74-79) */
    if (*k >= kend || meta[*k] != GG_META_BARRIER) return -1;
    const uint64_t stall = lat[(*k)++];
    if (!stall) { st[GG_IOCOOM_INSTRUCTIONS]--; return 0; }           /* released without a stall: no instruction */
    *curr += stall;
    st[GG_IOCOOM_SYNC_INSTRUCTIONS]++;                                /* core_model.cc:237-250 */
    st[GG_IOCOOM_SYNC_STALL_PS] += stall;
    return 0;
  }
  const uint64_t cost = lat_to_ps(in->cost, f);                       /* getCost (:70) */
  const uint64_t ready = *curr;                                       /* instruction_ready (:82-87) */
  const uint32_t nr = in->regs & 7u, nw = (in->regs >> 3) & 7u;
  if (nr + nw > 6) return -1;
  uint64_t rl = ready, re = ready;                                    /* :100-125 */
  for (uint32_t i = 0; i < nr; ++i) {
    const uint32_t r = in->reg[i];
    if (r >= GG_IOCOOM_NUM_REGISTERS) return -1;
    if (c->dep[r] == IO_LOAD_UNIT) rl = o_max(rl, c->sb[r]);
    else if (c->dep[r] == IO_EXECUTION_UNIT) re = o_max(re, c->sb[r]);
    else if (c->sb[r] > ready) return -1;
  }
  const uint64_t rr = o_max(rl, re);                                  /* :128-129 */
  uint64_t lqr = rr, rmr = rr;                                        /* :133-152 */
  for (uint32_t i = 0; i < (in->ops & 3u); ++i) {
    if (*k >= kend || meta[*k] == GG_META_BARRIER || (meta[*k] & GG_META_WRITE)) return -1;
    uint64_t comp;
    const uint64_t alloc = o_io_load(c, rr, addr[*k], lat[*k], &comp);
    st[GG_IOCOOM_DATA_ACCESSES]++; st[GG_IOCOOM_DATA_LATENCY_PS] += lat[*k];
    ++*k;
    lqr = o_max(lqr, alloc);
    rmr = o_max(rmr, comp);
  }
  const uint64_t wor = rmr + cost;                                    /* :158-166 */
  const int smov = (in->ops & GG_INS_SIMPLE_MOV_LOAD) != 0;
  for (uint32_t i = 0; i < nw; ++i) {                                 /* :172-184 */
    const uint32_t r = in->reg[nr + i];
    if (r >= GG_IOCOOM_NUM_REGISTERS) return -1;
    c->sb[r] = wor;
    c->dep[r] = smov ? IO_LOAD_UNIT : IO_EXECUTION_UNIT;
  }
  uint64_t sqr = wor;                                                 /* :186-201 */
  const uint32_t nwm = (in->ops >> 2) & 3u;
  for (uint32_t i = 0; i < nwm; ++i) {
    if (*k >= kend || meta[*k] == GG_META_BARRIER || !(meta[*k] & GG_META_WRITE)) return -1;
    const uint64_t alloc = o_io_store(c, wor, addr[*k], lat[*k]);
    st[GG_IOCOOM_DATA_ACCESSES]++; st[GG_IOCOOM_DATA_LATENCY_PS] += lat[*k];
    ++*k;
    sqr = o_max(sqr, alloc);
  }
  uint64_t mem = 0, ex = 0;                                           /* :209-252 */
  ex += re - ready;                       st[GG_IOCOOM_INTER_EXEC_STALL_PS] += re - ready;
  mem += rr - re;                         st[GG_IOCOOM_INTER_L1D_STALL_PS] += rr - re;
  mem += lqr - rr;                        st[GG_IOCOOM_LOAD_QUEUE_STALL_PS] += lqr - rr;
  *curr = lqr;
  if (!smov) {
    mem += rmr - lqr;                     st[GG_IOCOOM_INTRA_L1D_STALL_PS] += rmr - lqr;
    *curr = rmr;
    if (nwm > 0) {
      ex += wor - rmr;                    st[GG_IOCOOM_INTRA_EXEC_STALL_PS] += wor - rmr;
      mem += sqr - wor;                   st[GG_IOCOOM_STORE_QUEUE_STALL_PS] += sqr - wor;
      *curr = sqr;
    }
  }
  if (in->ops & GG_INS_ATOMIC) st[GG_IOCOOM_IMPLICIT_MFENCES]++;      /* updateMemoryFenceCounters (core_model.cc:221-235) */
  if (in->ops >> GG_INS_FENCE_SHIFT) st[GG_IOCOOM_EXPLICIT_FENCES]++;
  st[GG_IOCOOM_MEMORY_STALL_PS] += mem;                               /* core_model.cc:260-264 */
  st[GG_IOCOOM_EXECUTION_STALL_PS] += ex;
  return 0;
}

int oracle_iocoom(const gg_iocoom_params* p, const gg_ins* ins, const uint64_t* ins_offsets, const uint64_t* addr,
                  const uint32_t* meta, const uint64_t* lat, const uint64_t* acc_offsets, uint32_t tiles,
                  double frequency_ghz, uint64_t* stats)
{
  if (!p->num_load_queue_entries || p->num_load_queue_entries > IO_MAXQ || !p->num_store_queue_entries ||
      p->num_store_queue_entries > IO_MAXQ)
    return -1;
  o_iocoom* c = (o_iocoom*)malloc(sizeof(o_iocoom));
  if (!c) return -1;
  int bad = 0;
  for (uint32_t t = 0; t < tiles; ++t) {
    memset(c, 0, sizeof *c);                                          /* constructor (:10-45) */
    c->lq.n = p->num_load_queue_entries; c->lq.flag = p->speculative_loads_enabled != 0;
    c->sq.n = p->num_store_queue_entries; c->sq.flag = p->multiple_outstanding_RFOs_enabled != 0;
    for (uint32_t i = 0; i < IO_MAXQ; ++i) c->sq.addr[i] = ~0ull;     /* INVALID_ADDRESS (fixed_types.h:36) */
    c->one = lat_to_ps(1, frequency_ghz);
    uint64_t curr = 0, k = acc_offsets[t];
    for (uint64_t i = ins_offsets[t]; i < ins_offsets[t + 1] && !bad; ++i)
      bad = o_io_handle(c, &curr, &ins[i], addr, meta, lat, &k, acc_offsets[t + 1], frequency_ghz) != 0;
    if (k != acc_offsets[t + 1]) bad = 1;
    c->st[GG_IOCOOM_TIME_PS] = curr;
    memcpy(stats + (size_t)t * GG_NUM_IOCOOM_STATS, c->st, sizeof c->st);
    if (bad) break;
  }
  free(c);
  return bad ? -1 : 0;
}

/* ======================================================================== */
/* Cache (common/tile/memory_subsystem/cache/)                               */
/* ======================================================================== */
#define O_INVALID_TAG (~0ull)                        /* cache_line_info.h:21-22 */
enum { CS_I = GG_CSTATE_INVALID, CS_S = GG_CSTATE_SHARED, CS_M = GG_CSTATE_MODIFIED };

typedef struct { uint64_t tag; uint32_t cstate; uint32_t loc; } o_line;

typedef struct {
  uint32_t sets, ways, log_line, policy, write_back;
  o_line*   lines;     /* [sets][ways]   CacheSet::_cache_line_info_array     */
  uint8_t*  lru;       /* [sets][ways]   LRUReplacementPolicy::_lru_bits_vec  */
  uint32_t* rr;        /* [sets]         RoundRobin::_replacement_index_vec   */
  uint64_t  c[GG_NUM_CACHE_COUNTERS];
  /* miss-type tracking (track_miss_types, cache.cc:28-40,321-405): the
   * evicted / invalidated / fetched address sets as one map address -> 3 bits */
  int       track;
  uint64_t* mt_key;    /* open addressing, ~0 = empty                            */
  uint8_t*  mt_bits;   /* O_MT_EVICTED | O_MT_INVALIDATED | O_MT_FETCHED         */
  uint64_t  mt_cap, mt_n;
  uint64_t  mt[GG_NUM_MISS_TYPES];   /* _total_cold / capacity / sharing_misses */
} o_cache;
enum { O_MT_EVICTED = 1, O_MT_INVALIDATED = 2, O_MT_FETCHED = 4 };

static uint64_t o_mt_slot(const o_cache* c, uint64_t addr)
{
  uint64_t h = (addr >> 6) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  for (uint64_t i = h & (c->mt_cap - 1);; i = (i + 1) & (c->mt_cap - 1))
    if (c->mt_key[i] == addr || c->mt_key[i] == ~0ull) return i;
}
static uint8_t o_mt_get(const o_cache* c, uint64_t addr)
{
  if (!c->mt_cap) return 0;
  const uint64_t i = o_mt_slot(c, addr);
  return c->mt_key[i] == addr ? c->mt_bits[i] : 0;
}
static void o_mt_put(o_cache* c, uint64_t addr, uint8_t bits)
{
  if (2 * (c->mt_n + 1) > c->mt_cap) {               /* grow at half load */
    const uint64_t oc = c->mt_cap;
    uint64_t* ok = c->mt_key; uint8_t* ob = c->mt_bits;
    c->mt_cap = oc ? 2 * oc : 1024;
    c->mt_key = (uint64_t*)malloc(sizeof(uint64_t) * c->mt_cap);
    c->mt_bits = (uint8_t*)calloc(c->mt_cap, 1);
    for (uint64_t i = 0; i < c->mt_cap; ++i) c->mt_key[i] = ~0ull;
    for (uint64_t i = 0; i < oc; ++i)
      if (ok[i] != ~0ull) { const uint64_t j = o_mt_slot(c, ok[i]); c->mt_key[j] = ok[i]; c->mt_bits[j] = ob[i]; }
    free(ok); free(ob);
  }
  const uint64_t i = o_mt_slot(c, addr);
  if (c->mt_key[i] != addr) { c->mt_key[i] = addr; c->mt_n++; }
  c->mt_bits[i] = bits;
}
/* Cache::clearMissTypeTrackingSets (cache.cc:398-404): out of the first set
 * that holds the address, in the order evicted, invalidated, fetched */
static void o_mt_clear(o_cache* c, uint64_t addr)
{
  uint8_t b = o_mt_get(c, addr);
  if (b & O_MT_EVICTED) b &= (uint8_t)~O_MT_EVICTED;
  else if (b & O_MT_INVALIDATED) b &= (uint8_t)~O_MT_INVALIDATED;
  else if (b & O_MT_FETCHED) b &= (uint8_t)~O_MT_FETCHED;
  else return;
  o_mt_put(c, addr, b);
}
/* Cache::getMissType + updateMissTypeCounters (cache.cc:363-396) */
static void o_mt_classify(o_cache* c, uint64_t addr)
{
  const uint8_t b = o_mt_get(c, addr);
  if (b & O_MT_EVICTED) c->mt[GG_MT_CAPACITY]++;
  else if (b & (O_MT_INVALIDATED | O_MT_FETCHED)) c->mt[GG_MT_SHARING]++;
  else c->mt[GG_MT_COLD]++;
}

static void o_cache_init(o_cache* c, uint32_t size_kb, uint32_t assoc, uint32_t line,
                         uint32_t policy, uint32_t write_back)
{
  memset(c, 0, sizeof(*c));
  c->sets = size_kb * 1024u / (assoc * line);       /* cache.cc:44, cache_hash_fn.h:11 */
  c->ways = assoc;
  c->log_line = (uint32_t)floor_log2(line);
  c->policy = policy;
  c->write_back = write_back;
  c->lines = (o_line*)malloc(sizeof(o_line) * c->sets * c->ways);
  c->lru = (uint8_t*)malloc((size_t)c->sets * c->ways);
  c->rr = (uint32_t*)malloc(sizeof(uint32_t) * c->sets);
  for (uint32_t s = 0; s < c->sets; ++s) {
    for (uint32_t w = 0; w < c->ways; ++w) {
      o_line* l = &c->lines[(size_t)s * c->ways + w];
      l->tag = O_INVALID_TAG; l->cstate = CS_I; l->loc = GG_LOC_INVALID;
      c->lru[(size_t)s * c->ways + w] = (uint8_t)w;  /* lru_replacement_policy.cc:5-18 */
    }
    c->rr[s] = c->ways - 1;                         /* round_robin_replacement_policy.cc:4-9 */
  }
}

static void o_cache_free(o_cache* c) { free(c->lines); free(c->lru); free(c->rr); free(c->mt_key); free(c->mt_bits); }

/* cache_hash_fn.h:17-18 and Cache::getTag (cache.cc:495-498) */
static uint32_t o_set(const o_cache* c, uint64_t addr) { return (uint32_t)((addr >> c->log_line) & (c->sets - 1)); }
static uint64_t o_tag(const o_cache* c, uint64_t addr) { return addr >> c->log_line; }

/* CacheSet::find — scans ways from high to low (cache_set.cc:57-70) */
static int o_find(const o_cache* c, uint32_t set, uint64_t tag)
{
  for (int w = (int)c->ways - 1; w >= 0; --w)
    if (c->lines[(size_t)set * c->ways + w].tag == tag) return w;
  return -1;
}

/* LRUReplacementPolicy::update (lru_replacement_policy.cc:40-50); RR update is a no-op */
static void o_policy_update(o_cache* c, uint32_t set, uint32_t way)
{
  if (c->policy != GG_POLICY_LRU) return;
  uint8_t* b = &c->lru[(size_t)set * c->ways];
  uint8_t acc = b[way];
  for (uint32_t i = 0; i < c->ways; ++i) if (b[i] < acc) b[i]++;
  b[way] = 0;
}

/* getReplacementWay: LRU (lru_replacement_policy.cc:23-38), RR (round_robin_replacement_policy.cc:13-22) */
static int o_victim(o_cache* c, uint32_t set)
{
  if (c->policy == GG_POLICY_LRU) {
    const uint8_t* b = &c->lru[(size_t)set * c->ways];
    uint32_t way = c->ways;
    for (uint32_t i = 0; i < c->ways; ++i) {
      if (c->lines[(size_t)set * c->ways + i].tag == O_INVALID_TAG) return (int)i;
      else if (b[i] == c->ways - 1) way = i;
    }
    return (way < c->ways) ? (int)way : -1;          /* LOG_ASSERT_ERROR "Error Finding LRU bits" */
  }
  uint32_t cur = c->rr[set];
  c->rr[set] = (c->rr[set] == 0) ? (c->ways - 1) : (c->rr[set] - 1);
  return (int)cur;
}

/* Cache::updateMissCounters (cache.cc:321-360), with the miss type when tracked */
static void o_update_miss_counters(o_cache* c, uint64_t addr, int is_write, int miss)
{
  c->c[GG_CC_ACCESSES]++;
  if (!is_write) c->c[GG_CC_READ_ACCESSES]++; else c->c[GG_CC_WRITE_ACCESSES]++;
  if (miss) {
    c->c[GG_CC_MISSES]++;
    if (!is_write) c->c[GG_CC_READ_MISSES]++; else c->c[GG_CC_WRITE_MISSES]++;
    if (c->track) o_mt_classify(c, addr);
  }
}

/* Cache::accessCacheLine (cache.cc:84-112): find (must hit), read/write_line -> policy update */
static int o_access_line(o_cache* c, uint64_t addr, int is_store)
{
  uint32_t s = o_set(c, addr);
  int w = o_find(c, s, o_tag(c, addr));
  if (w < 0) return GG_ERR_STATE;                    /* LOG_ASSERT_ERROR(cache_line_info) */
  o_policy_update(c, s, (uint32_t)w);                /* cache_set.cc:31-55 */
  c->c[is_store ? GG_CC_DATA_WRITES : GG_CC_DATA_READS]++;
  return 0;
}

/* Cache::insertCacheLine (cache.cc:114-184) + CacheSet::insert (cache_set.cc:72-103) */
static int o_insert_line(o_cache* c, uint64_t addr, const o_line* in, int* eviction,
                         uint64_t* evicted_addr, o_line* evicted)
{
  uint32_t s = o_set(c, addr);
  int w = o_victim(c, s);
  if (w < 0 || (uint32_t)w >= c->ways) return GG_ERR_STATE;
  o_line* l = &c->lines[(size_t)s * c->ways + w];
  if (l->tag != O_INVALID_TAG) { *eviction = 1; *evicted = *l; }
  else *eviction = 0;                                /* evicted keeps the caller's default */
  *l = *in;
  o_policy_update(c, s, (uint32_t)w);
  *evicted_addr = evicted->tag << c->log_line;       /* getAddressFromTag (cache.cc:514-518) */
  if (c->track) {                                    /* cache.cc:131-148 */
    if (*eviction) o_mt_put(c, *evicted_addr, (uint8_t)(o_mt_get(c, *evicted_addr) | O_MT_EVICTED));
    o_mt_clear(c, addr);
    o_mt_put(c, addr, (uint8_t)(o_mt_get(c, addr) | O_MT_FETCHED));
  }
  if (*eviction) {
    c->c[GG_CC_TAG_READS]++; c->c[GG_CC_DATA_READS]++;
    c->c[GG_CC_EVICTIONS]++;
    if (c->write_back && (evicted->cstate == CS_M || evicted->cstate == GG_CSTATE_OWNED))  /* CacheState::dirty(): M/O/DIRTY */
      c->c[GG_CC_DIRTY_EVICTIONS]++;
  } else {
    c->c[GG_CC_TAG_READS]++;
  }
  c->c[GG_CC_TAG_WRITES]++; c->c[GG_CC_DATA_WRITES]++;
  return 0;
}

/* Cache::getCacheLineInfo (cache.cc:187-215): out keeps the caller's default when absent */
static void o_get_line_info(o_cache* c, uint64_t addr, o_line* out)
{
  uint32_t s = o_set(c, addr);
  int w = o_find(c, s, o_tag(c, addr));
  if (w >= 0) *out = c->lines[(size_t)s * c->ways + w];
  c->c[GG_CC_TAG_READS]++;
}

/* Cache::setCacheLineInfo (cache.cc:218-241) */
static int o_set_line_info(o_cache* c, uint64_t addr, const o_line* in)
{
  uint32_t s = o_set(c, addr);
  int w = o_find(c, s, o_tag(c, addr));
  if (w < 0) return GG_ERR_STATE;
  if (c->track && in->cstate == CS_I)                /* cache.cc:228-230 */
    o_mt_put(c, addr, (uint8_t)(o_mt_get(c, addr) | O_MT_INVALIDATED));
  c->lines[(size_t)s * c->ways + w] = *in;
  c->c[GG_CC_TAG_WRITES]++;
  return 0;
}

static o_line o_default_line(void) { o_line l = { O_INVALID_TAG, CS_I, GG_LOC_INVALID }; return l; }
static int cs_readable(uint32_t s) { return s == CS_M || s == 3 || s == 2 || s == CS_S; } /* cache_state.h:26-29 */
static int cs_writable(uint32_t s) { return s == CS_M || s == 3; }                         /* cache_state.h:30-33 */

/* ======================================================================== */
/* pr_l1_pr_l2_dram_directory_msi controllers, private (decoupled) mode      */
/* ======================================================================== */
typedef struct { o_cache l1, l2; } o_tile;

struct oracle_cache { gg_config cfg; uint32_t ntiles; o_tile* t; };

oracle_cache* oracle_cache_create(const gg_config* cfg)
{
  oracle_cache* oc = (oracle_cache*)calloc(1, sizeof(*oc));
  oc->cfg = *cfg;
  oc->ntiles = cfg->num_tiles;
  oc->t = (o_tile*)calloc(cfg->num_tiles, sizeof(o_tile));
  for (uint32_t i = 0; i < cfg->num_tiles; ++i) {
    /* L1-D is WRITE_THROUGH (l1_cache_cntlr.cc:55-71), L2 WRITE_BACK (l2_cache_cntlr.cc:31-46) */
    o_cache_init(&oc->t[i].l1, cfg->l1d_size_kb, cfg->l1d_assoc, cfg->line_size, cfg->l1d_policy, 0);
    o_cache_init(&oc->t[i].l2, cfg->l2_size_kb, cfg->l2_assoc, cfg->line_size, cfg->l2_policy, 1);
    oc->t[i].l1.track = cfg->l1i_track_miss_types != 0;   /* the L1-D takes the L1-I flag (l1_cache_cntlr.cc:69) */
    oc->t[i].l2.track = cfg->l2_track_miss_types != 0;
  }
  return oc;
}

void oracle_cache_destroy(oracle_cache* oc)
{
  if (!oc) return;
  for (uint32_t i = 0; i < oc->ntiles; ++i) { o_cache_free(&oc->t[i].l1); o_cache_free(&oc->t[i].l2); }
  free(oc->t); free(oc);
}

/* L1CacheCntlr::invalidateCacheLine (l1_cache_cntlr.cc:293-305); returns 1 if a valid line was invalidated */
static int l1_invalidate(o_tile* T, uint64_t addr, int* err)
{
  o_line info = o_default_line();
  o_get_line_info(&T->l1, addr, &info);
  if (info.tag != O_INVALID_TAG) {
    info.tag = O_INVALID_TAG; info.cstate = CS_I;     /* CacheLineInfo::invalidate (cache_line_info.cc:39-43) */
    if (o_set_line_info(&T->l1, addr, &info)) *err = 1;
    return 1;
  }
  return 0;
}

/* L1CacheCntlr::accessCache (l1_cache_cntlr.cc:182-205) incl. the write-through to L2 */
static void l1_access_cache(o_tile* T, uint64_t addr, int is_write, int* err)
{
  if (o_access_line(&T->l1, addr, is_write)) *err = 1;
  if (is_write && o_access_line(&T->l2, addr, 1)) *err = 1;   /* L2CacheCntlr::writeCacheLine (l2:66-70) */
}

/* L2CacheCntlr::insertCacheLineInL1 (l2_cache_cntlr.cc:133-165) */
static void l2_insert_in_l1(o_tile* T, uint64_t addr, uint32_t cstate, uint32_t* res, int* err)
{
  o_line in = { o_tag(&T->l1, addr), cstate, GG_LOC_INVALID };   /* l1_cache_cntlr.cc:245-261 */
  o_line ev = o_default_line();
  int eviction = 0; uint64_t ev_addr = 0;
  if (o_insert_line(&T->l1, addr, &in, &eviction, &ev_addr, &ev)) { *err = 1; return; }
  if (eviction) {
    *res |= GG_RES_L1_EVICT;
    o_line l2i = o_default_line();
    o_get_line_info(&T->l2, ev_addr, &l2i);
    if (l2i.loc != GG_LOC_L1D) { *err = 1; return; }  /* LOG_ASSERT_ERROR: mem_component is L1-D */
    l2i.loc = GG_LOC_INVALID;                          /* clearCachedLoc */
    if (o_set_line_info(&T->l2, ev_addr, &l2i)) *err = 1;
  }
}

/* L2CacheCntlr::insertCacheLine (l2_cache_cntlr.cc:74-116) */
static void l2_insert(o_tile* T, uint64_t addr, uint32_t cstate, uint32_t* res, uint64_t* evicted_out, int* err)
{
  o_line in = { o_tag(&T->l2, addr), cstate, GG_LOC_L1D };
  o_line ev = o_default_line();
  int eviction = 0; uint64_t ev_addr = 0;
  if (o_insert_line(&T->l2, addr, &in, &eviction, &ev_addr, &ev)) { *err = 1; return; }
  if (eviction) {
    *res |= GG_RES_L2_EVICT;
    *evicted_out = ev_addr;
    if (ev.loc != GG_LOC_INVALID)                      /* invalidateCacheLineInL1 (l2:124-131) */
      if (l1_invalidate(T, ev_addr, err)) *res |= GG_RES_L2_EVICT_INV_L1;
    if (ev.cstate == CS_M) *res |= GG_RES_L2_EVICT_DIRTY;       /* FLUSH_REP + data */
    else if (ev.cstate != CS_S) *err = 1;                        /* LOG_ASSERT_ERROR(SHARED) -> INV_REP */
  }
}

/*
 * One line access of tile T in private mode: L1CacheCntlr::processMemOpFromCore
 * (l1_cache_cntlr.cc:89-180) with the directory granting every request
 * (DramDirectoryCntlr::processEx/ShReqFromL2Cache on an UNCACHED entry,
 * dram_directory_cntlr.cc:238-380: EX_REQ -> EX_REP/MODIFIED, SH_REQ -> SH_REP/SHARED).
 */
static uint32_t modep_access(o_tile* T, uint64_t addr, int is_write, uint64_t* evicted_out, int* err)
{
  uint32_t res = 0;
  *evicted_out = ~0ull;
  for (int access_num = 1; access_num <= 2; ++access_num) {
    /* operationPermissibleinL1Cache (l1:207-243) */
    o_line info = o_default_line();
    o_get_line_info(&T->l1, addr, &info);
    int hit = is_write ? cs_writable(info.cstate) : cs_readable(info.cstate);
    if (access_num == 1) o_update_miss_counters(&T->l1, addr, is_write, !hit);
    if (hit) { l1_access_cache(T, addr, is_write, err); return res; }
    if (access_num == 2) { *err = 1; return res; }   /* LOG_ASSERT_ERROR(access_num == 1 || 2) */
    res |= GG_RES_L1_MISS;

    if (l1_invalidate(T, addr, err)) res |= GG_RES_L1_INVAL;   /* l1:135-137 */

    /* L2CacheCntlr::processShmemRequestFromL1Cache (l2:180-224) */
    o_line l2i = o_default_line();
    o_get_line_info(&T->l2, addr, &l2i);
    uint32_t cstate = l2i.cstate;
    int l2hit = is_write ? cs_writable(cstate) : cs_readable(cstate);  /* l2:504-527 */
    o_update_miss_counters(&T->l2, addr, is_write, !l2hit);
    if (l2hit) {
      if (o_access_line(&T->l2, addr, 0)) *err = 1;   /* readCacheLine */
      l2_insert_in_l1(T, addr, cstate, &res, err);
      l2i.loc = GG_LOC_L1D;                          /* setCachedLoc / setForcedCachedLoc */
      if (o_set_line_info(&T->l2, addr, &l2i)) *err = 1;
      l1_access_cache(T, addr, is_write, err);       /* l1:145-159 */
      return res;
    }

    /* L2 miss: handleMsgFromL1Cache (l2:226-258) */
    res |= GG_RES_L2_MISS;
    uint32_t new_state;
    if (is_write) {                                  /* processExReqFromL1Cache (l2:260-282) */
      o_line x = o_default_line();
      o_get_line_info(&T->l2, addr, &x);
      if (x.cstate == CS_S) {
        x.tag = O_INVALID_TAG; x.cstate = CS_I; x.loc = GG_LOC_INVALID;  /* PrL2CacheLineInfo::invalidate */
        if (o_set_line_info(&T->l2, addr, &x)) *err = 1;
        res |= GG_RES_UPGRADE;                       /* INV_REP then EX_REQ to the home */
      } else if (x.cstate != CS_I) *err = 1;
      new_state = CS_M;                              /* EX_REP */
    } else {
      new_state = CS_S;                              /* processShReqFromL1Cache -> SH_REP */
    }
    /* insertCacheLineInHierarchy (l2:167-178) */
    l2_insert(T, addr, new_state, &res, evicted_out, err);
    l2_insert_in_l1(T, addr, new_state, &res, err);
  }
  return res;
}

int oracle_cache_run(oracle_cache* oc, const uint64_t* addr, const uint32_t* meta,
                     const uint64_t* tile_offsets, uint32_t tile_begin, uint32_t tile_end,
                     uint32_t* result, uint64_t* evicted)
{
  int err = 0;
  const uint64_t line_mask = ~((uint64_t)oc->cfg.line_size - 1);
  for (uint32_t t = tile_begin; t < tile_end && t < oc->ntiles; ++t) {
    o_tile* T = &oc->t[t];
    for (uint64_t i = tile_offsets[t]; i < tile_offsets[t + 1]; ++i) {
      uint64_t ev = ~0ull;
      uint32_t r = modep_access(T, addr[i] & line_mask, (int)(meta[i] & GG_META_WRITE), &ev, &err);
      if (result) result[i] = r;
      if (evicted) evicted[i] = ev;
    }
  }
  return err ? GG_ERR_STATE : 0;
}

void oracle_cache_counters(const oracle_cache* oc, uint64_t* out)
{
  for (uint32_t t = 0; t < oc->ntiles; ++t) {
    memcpy(out + ((size_t)t * 2 + 0) * GG_NUM_CACHE_COUNTERS, oc->t[t].l1.c, sizeof(uint64_t) * GG_NUM_CACHE_COUNTERS);
    memcpy(out + ((size_t)t * 2 + 1) * GG_NUM_CACHE_COUNTERS, oc->t[t].l2.c, sizeof(uint64_t) * GG_NUM_CACHE_COUNTERS);
  }
}

void oracle_cache_miss_types(const oracle_cache* oc, uint64_t* out)
{
  for (uint32_t t = 0; t < oc->ntiles; ++t) {
    memcpy(out + ((size_t)t * 2 + 0) * GG_NUM_MISS_TYPES, oc->t[t].l1.mt, sizeof(uint64_t) * GG_NUM_MISS_TYPES);
    memcpy(out + ((size_t)t * 2 + 1) * GG_NUM_MISS_TYPES, oc->t[t].l2.mt, sizeof(uint64_t) * GG_NUM_MISS_TYPES);
  }
}

static o_cache* oc_level(oracle_cache* oc, uint32_t tile, int level)
{
  if (tile >= oc->ntiles) return NULL;
  return level == GG_L1D ? &oc->t[tile].l1 : &oc->t[tile].l2;
}

int oracle_cache_get_line_info(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, gg_line_info* out)
{
  o_cache* c = oc_level(oc, tile, level);
  if (!c) return GG_ERR_INVALID;
  o_line l = { out->tag, out->cstate, out->cached_loc };
  o_get_line_info(c, addr, &l);
  out->tag = l.tag; out->cstate = l.cstate; out->cached_loc = l.loc;
  return 0;
}

int oracle_cache_set_line_info(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, const gg_line_info* in)
{
  o_cache* c = oc_level(oc, tile, level);
  if (!c) return GG_ERR_INVALID;
  o_line l = { in->tag, in->cstate, level == GG_L2 ? in->cached_loc : GG_LOC_INVALID };
  return o_set_line_info(c, addr, &l);
}

int oracle_cache_access_line(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, int is_store)
{
  o_cache* c = oc_level(oc, tile, level);
  if (!c) return GG_ERR_INVALID;
  return o_access_line(c, addr, is_store);
}

int oracle_cache_insert_line(oracle_cache* oc, uint32_t tile, int level, uint64_t addr,
                             const gg_line_info* in, int* eviction, uint64_t* evicted_addr,
                             gg_line_info* evicted_info)
{
  o_cache* c = oc_level(oc, tile, level);
  if (!c) return GG_ERR_INVALID;
  o_line l = { in->tag, in->cstate, level == GG_L2 ? in->cached_loc : GG_LOC_INVALID };
  o_line ev = { evicted_info->tag, evicted_info->cstate, evicted_info->cached_loc };
  int rc = o_insert_line(c, addr, &l, eviction, evicted_addr, &ev);
  evicted_info->tag = ev.tag; evicted_info->cstate = ev.cstate; evicted_info->cached_loc = ev.loc;
  return rc;
}

/* ======================================================================== */
/* IntervalTree (common/misc/interval_tree.cc:40-394)                        */
/* ======================================================================== */
typedef struct {
  int parent, left, right;     /* node indices, -1 = NULL */
  int32_t height;
  uint64_t key, first, second; /* key == interval.first always */
} it_node;

typedef struct { it_node* n; int root; uint32_t size; } itree;

static int32_t it_h(const itree* t, int x) { return x < 0 ? 0 : t->n[x].height; }

/* updateChildPointer (interval_tree.cc:45-72): dir 0 = INVALID (by key), 1 = LEFT, 2 = RIGHT */
static void it_upd_child(itree* t, int node, int child, int dir)
{
  if (node < 0) return;
  if (dir == 0) {
    if (t->n[node].key < t->n[child].key) t->n[node].right = child; else t->n[node].left = child;
  } else if (dir == 1) t->n[node].left = child;
  else t->n[node].right = child;
}

/* updateParentPointer (interval_tree.cc:74-81) */
static void it_upd_parent(itree* t, int node, int parent)
{
  if (node >= 0) t->n[node].parent = parent;
  if (parent < 0) t->root = node;
}

static int it_balanced(const itree* t, int x) { return abs(it_h(t, t->n[x].left) - it_h(t, t->n[x].right)) <= 1; }
static void it_upd_height(itree* t, int x)
{
  int32_t a = it_h(t, t->n[x].left), b = it_h(t, t->n[x].right);
  t->n[x].height = (a > b ? a : b) + 1;
}

/* performRotation (interval_tree.cc:103-140): cw = CLOCKWISE */
static void it_rotate(itree* t, int y, int cw)
{
  int x;
  if (cw) {
    x = t->n[y].left;
    it_upd_parent(t, x, t->n[y].parent);
    it_upd_child(t, t->n[x].parent, x, 0);
    t->n[y].left = t->n[x].right;
    it_upd_parent(t, t->n[y].left, y);
    t->n[x].right = y;
    it_upd_parent(t, y, x);
  } else {
    x = t->n[y].right;
    it_upd_parent(t, x, t->n[y].parent);
    it_upd_child(t, t->n[x].parent, x, 0);
    t->n[y].right = t->n[x].left;
    it_upd_parent(t, t->n[y].right, y);
    t->n[x].left = y;
    it_upd_parent(t, y, x);
  }
  it_upd_height(t, y);
  it_upd_height(t, x);
}

/* balanceHeight (interval_tree.cc:142-197) */
static int it_balance(itree* t, int z)
{
  int zl = t->n[z].left, zr = t->n[z].right;
  int y_left = it_h(t, zl) > it_h(t, zr);
  int y = y_left ? zl : zr;
  int yl = t->n[y].left, yr = t->n[y].right;
  int x, x_left;
  if (it_h(t, yl) != it_h(t, yr)) { x_left = it_h(t, yl) > it_h(t, yr); x = x_left ? yl : yr; }
  else if (y_left) { x = yl; x_left = 1; }
  else { x = yr; x_left = 0; }
  if (y_left) {
    if (!x_left) { it_rotate(t, y, 0); it_rotate(t, z, 1); return x; }
    it_rotate(t, z, 1); return y;
  } else {
    if (x_left) { it_rotate(t, y, 1); it_rotate(t, z, 0); return x; }
    it_rotate(t, z, 0); return y;
  }
}

/* rebalanceAVLTree (interval_tree.cc:199-229) */
static void it_rebalance(itree* t, int r)
{
  while (r >= 0) {
    int32_t old = t->n[r].height;
    int nr = r;
    if (!it_balanced(t, r)) nr = it_balance(t, r);
    else it_upd_height(t, r);
    if (t->n[nr].height == old) return;
    r = t->n[nr].parent;
  }
}

/* insert / insertInTree (interval_tree.cc:250-290) */
static int it_insert(itree* t, int node)
{
  t->size++;
  int r = t->root;
  for (;;) {
    if (t->n[node].key < t->n[r].key) {
      if (t->n[r].left >= 0) r = t->n[r].left;
      else { t->n[r].left = node; t->n[node].parent = r; it_rebalance(t, r); return 0; }
    } else if (t->n[node].key > t->n[r].key) {
      if (t->n[r].right >= 0) r = t->n[r].right;
      else { t->n[r].right = node; t->n[node].parent = r; it_rebalance(t, r); return 0; }
    } else return GG_ERR_STATE;                   /* "Found 2 nodes with same key" */
  }
}

/* findMinKeyNode (interval_tree.cc:241-248) */
static int it_min(const itree* t, int r) { while (t->n[r].left >= 0) r = t->n[r].left; return r; }

/* removeFromTree (interval_tree.cc:300-340): returns the node slot to release */
static int it_remove_rec(itree* t, int node)
{
  it_node* n = &t->n[node];
  if (n->left < 0) {
    if (n->parent >= 0)
      it_upd_child(t, n->parent, n->right, (t->n[n->parent].key < n->key) ? 2 : 1);
    it_upd_parent(t, n->right, n->parent);
    it_rebalance(t, n->parent);
    return node;
  } else if (n->right < 0) {
    it_upd_child(t, n->parent, n->left, 0);
    it_upd_parent(t, n->left, n->parent);
    it_rebalance(t, n->parent);
    return node;
  } else {
    int succ = it_min(t, n->right);
    it_remove_rec(t, succ);
    /* swap key/interval of node and successor (interval_tree.cc:231-239) */
    it_node tmp = t->n[node];
    t->n[node].key = t->n[succ].key; t->n[node].first = t->n[succ].first; t->n[node].second = t->n[succ].second;
    t->n[succ].key = tmp.key; t->n[succ].first = tmp.first; t->n[succ].second = tmp.second;
    return succ;
  }
}
static int it_remove(itree* t, int node) { t->size--; return it_remove_rec(t, node); }

/* searchTree (interval_tree.cc:349-377) */
static int it_search(const itree* t, uint64_t a, uint64_t b, int r)
{
  while (r >= 0) {
    const it_node* n = &t->n[r];
    if (a >= n->first && b <= n->second) return r;
    if (b < n->first) {
      int f = it_search(t, a, b, n->left);
      if (f >= 0) return f;
    }
    if (a < n->first && (n->second - n->first) >= (b - a)) return r;
    r = n->right;
  }
  return -1;
}

/* ======================================================================== */
/* QueueModelMG1 (shared_models/queue_models/queue_model_m_g_1.cc:18-56)     */
/* ======================================================================== */
typedef struct { double sig_sq, sig; uint64_t n, newest; } mg1;

static double sq(double x) { return x * x; }
static uint64_t mg1_delay(const mg1* m)
{
  if (m->n == 0) return 0;
  double variance = (m->sig_sq / m->n) - sq(m->sig / m->n);
  double service_rate = 1.0 / (m->sig / m->n);
  double arrival_rate = ((double)m->n) / m->newest;
  if (arrival_rate >= service_rate) arrival_rate = 0.999 * service_rate;
  return (uint64_t)ceil(0.5 * service_rate * arrival_rate * ((1 / sq(service_rate)) + variance) /
                        (service_rate - arrival_rate));
}
static void mg1_update(mg1* m, uint64_t t, uint64_t s, uint64_t w)
{
  m->sig_sq += sq((double)s);
  m->sig += s;
  m->n++;
  uint64_t x = t + w + s;
  m->newest = (m->newest > x) ? m->newest : x;
}

/* ======================================================================== */
/* QueueModelHistoryTree (queue_model_history_tree.cc:14-167)                */
/* ======================================================================== */
struct oracle_htree {
  uint64_t min_proc;
  int max_size, analytical;
  itree t;
  int* free_list; int free_tail;                  /* allocateMemory (:129-137) */
  mg1 m;
  uint64_t analytical_requests;
  uint64_t util_cycles, last_req, total_req;      /* queue_model.cc:41-55 */
  /* QueueModel::create (queue_model.cc:19-39) picks the model by type */
  uint32_t type;                                  /* GG_QM_* */
  /* history_list (queue_model_history_list.cc): the free-interval std::list
   * as an array in list order, room for max_list_size + 1 entries (the list
   * overgrows by one before its front is dropped, :128-131) */
  uint64_t (*lst)[2]; uint32_t lsize; int interleaving;
  /* basic (queue_model_basic.cc) with MovingAverage<UInt64> (moving_average.h) */
  uint64_t queue_time;
  int avg;                                        /* GG_MAVG_* */
  uint32_t win_max, front, back;                  /* ModuloNum(window + 1) */
  uint64_t* win;
  double mean;
};

static int ht_alloc(oracle_htree* h, uint64_t a, uint64_t b)    /* allocateNode (:146-157) */
{
  if (h->free_tail < 0) return -1;
  int idx = h->free_list[h->free_tail--];
  it_node* n = &h->t.n[idx];
  n->parent = n->left = n->right = -1; n->height = 1; n->key = a; n->first = a; n->second = b;
  return idx;
}
static void ht_release(oracle_htree* h, int idx) { h->free_list[++h->free_tail] = idx; } /* :159-167 */

oracle_htree* oracle_htree_create(uint64_t min_proc, int max_list_size, int analytical)
{
  oracle_htree* h = (oracle_htree*)calloc(1, sizeof(*h));
  h->min_proc = min_proc; h->max_size = max_list_size; h->analytical = analytical;
  h->t.n = (it_node*)calloc((size_t)max_list_size, sizeof(it_node));
  h->free_list = (int*)malloc(sizeof(int) * (size_t)max_list_size);
  for (int i = 0; i < max_list_size; ++i) h->free_list[i] = i;
  h->free_tail = max_list_size - 1;
  h->t.root = ht_alloc(h, 0, UINT64_MAX);         /* PAIR(0, UINT64_MAX) (:30) */
  h->t.size = 1;
  return h;
}

/* QueueModelHistoryList(min_processing_time) (queue_model_history_list.cc:9-28) */
static oracle_htree* qm_list_create(uint64_t min_proc, int max_list_size, int analytical, int interleaving)
{
  oracle_htree* h = (oracle_htree*)calloc(1, sizeof(*h));
  h->type = GG_QM_HISTORY_LIST;
  h->min_proc = min_proc; h->max_size = max_list_size; h->analytical = analytical;
  h->interleaving = interleaving;
  h->lst = (uint64_t(*)[2])calloc((size_t)max_list_size + 2, sizeof(*h->lst));
  h->lst[0][0] = 0; h->lst[0][1] = UINT64_MAX;    /* push_back(make_pair(0, UINT64_MAX)) (:26) */
  h->lsize = 1;
  return h;
}

/* QueueModelBasic (queue_model_basic.cc:7-28): moving_avg_window_size / _type */
static oracle_htree* qm_basic_create(uint32_t window, int avg)
{
  oracle_htree* h = (oracle_htree*)calloc(1, sizeof(*h));
  h->type = GG_QM_BASIC;
  h->avg = avg;
  h->win_max = window;
  h->win = (uint64_t*)calloc((size_t)window + 1, sizeof(uint64_t));   /* _num_list.resize(max + 1) */
  return h;
}

oracle_htree* oracle_qmodel_create(uint32_t type, uint32_t aux, uint64_t min_proc, int max_list_size, int analytical)
{
  if (type == GG_QM_HISTORY_LIST) return qm_list_create(min_proc, max_list_size, analytical, aux == 0);
  if (type == GG_QM_BASIC) {
    const uint32_t w = (aux & 0xFFFFu) ? (aux & 0xFFFFu) : 64u;
    return qm_basic_create(w, (int)(aux >> 16));
  }
  return oracle_htree_create(min_proc, max_list_size, analytical);
}

void oracle_htree_destroy(oracle_htree* h) { if (h) { free(h->t.n); free(h->free_list); free(h->lst); free(h->win); free(h); } }
uint64_t oracle_htree_analytical_requests(const oracle_htree* h) { return h->analytical_requests; }
uint32_t oracle_htree_size(const oracle_htree* h) { return h->t.size; }

/* ---- history list: std::list operations on the array (index = iterator) ---- */
static void lst_erase(oracle_htree* h, uint32_t i)
{
  memmove(&h->lst[i], &h->lst[i + 1], sizeof(*h->lst) * (h->lsize - i - 1));
  h->lsize--;
}
static void lst_insert(oracle_htree* h, uint32_t i, uint64_t a, uint64_t b)   /* insert before i */
{
  memmove(&h->lst[i + 1], &h->lst[i], sizeof(*h->lst) * (h->lsize - i));
  h->lst[i][0] = a; h->lst[i][1] = b;
  h->lsize++;
}

/* computeUsingHistoryList (queue_model_history_list.cc:68-134) */
static uint64_t list_delay(oracle_htree* h, uint64_t t, uint64_t p)
{
  uint64_t qd = 0;
  const uint64_t mp = h->min_proc;
  for (uint32_t it = 0; it < h->lsize; ++it) {
    const uint64_t a = h->lst[it][0], b = h->lst[it][1];
    if (t >= a && (t + p) <= b) {                 /* fits: no additional delay */
      lst_erase(h, it);
      if ((t - a) >= mp) lst_insert(h, it++, a, t);
      if ((b - (t + p)) >= mp) lst_insert(h, it++, t + p, b);
      break;
    } else if (t < a && (a + p) <= b) {           /* starts at the interval */
      qd += a - t;
      lst_erase(h, it);
      if ((b - (a + p)) >= mp) lst_insert(h, it, a + p, b);
      break;
    } else if (h->interleaving) {
      if (t >= a && t < b) {
        lst_erase(h, it);
        if ((t - a) >= mp) lst_insert(h, it++, a, t);
        it--;                                     /* the loop's ++ lands after the erased interval */
        t = b;
        p -= (b - t);                             /* the reference subtracts after moving pkt_time: 0 */
      } else if (t < a) {
        lst_erase(h, it);
        it--;
        qd += a - t;
        t = b;
        p -= (b - a);
      }
    }
  }
  if (h->lsize > (uint32_t)h->max_size) lst_erase(h, 0);
  return qd;
}

/* MovingAverage<UInt64>::compute (moving_average.h): arithmetic mean / median */
static uint64_t mavg(oracle_htree* h, uint64_t x)
{
  const uint32_t M = h->win_max + 1;
  const uint32_t cws = (h->back >= h->front) ? h->back - h->front : h->back + M - h->front;
  uint64_t r;
  if (h->avg == GG_MAVG_MEDIAN) {
    h->win[h->back] = x;                          /* addToWindow */
    h->back = (h->back + 1) % M;
    if (h->back == h->front) h->front = (h->front + 1) % M;
    const uint32_t c2 = (h->back >= h->front) ? h->back - h->front : h->back + M - h->front;
    r = h->win[(h->front + (c2 / 2) % M) % M];
  } else {                                        /* MovingArithmeticMean */
    if (cws == h->win_max) {
      const uint64_t old = h->win[h->front];
      h->mean += (((double)x / cws) - ((double)old / cws));
    } else {
      h->mean = (h->mean * cws + x) / (cws + 1);
    }
    h->win[h->back] = x;
    h->back = (h->back + 1) % M;
    if (h->back == h->front) h->front = (h->front + 1) % M;
    r = (uint64_t)h->mean;
  }
  return r;
}

/* QueueModelBasic::computeQueueDelay (queue_model_basic.cc:34-61) */
static uint64_t basic_delay(oracle_htree* h, uint64_t t, uint64_t p)
{
  const uint64_t ref = (h->avg == GG_MAVG_NONE) ? t : mavg(h, t);
  const uint64_t qd = (h->queue_time > ref) ? (h->queue_time - ref) : 0;
  h->queue_time = ((h->queue_time > ref) ? h->queue_time : ref) + p;
  h->util_cycles += p;
  if (ref + qd + p > h->last_req) h->last_req = ref + qd + p;
  h->total_req++;
  return qd;
}

/* computeQueueDelay (queue_model_history_tree.cc:44-126; history_list: queue_model_history_list.cc:40-66) */
uint64_t oracle_htree_delay(oracle_htree* h, uint64_t t, uint64_t p)
{
  uint64_t qd = UINT64_MAX;
  if (h->type == GG_QM_BASIC) return basic_delay(h, t, p);
  if (h->type == GG_QM_HISTORY_LIST) {
    if (h->analytical && ((t + p) < h->lst[0][0])) {
      h->analytical_requests++;
      qd = mg1_delay(&h->m);
    } else {
      qd = list_delay(h, t, p);
    }
    mg1_update(&h->m, t, p, qd);
    h->util_cycles += p;
    if (t + qd + p > h->last_req) h->last_req = t + qd + p;
    h->total_req++;
    return qd;
  }
  itree* T = &h->t;
  int min_node = it_search(T, 0, 1, T->root);
  if (T->size >= (uint32_t)h->max_size) ht_release(h, it_remove(T, min_node));
  min_node = it_search(T, 0, 1, T->root);
  if (h->analytical && (T->n[min_node].first > (t + p))) {
    h->analytical_requests++;
    qd = mg1_delay(&h->m);
  } else {
    int node = it_search(T, t, t + p, T->root);
    if (node < 0) return UINT64_MAX;              /* LOG_PRINT_ERROR("node = (NULL)") */
    it_node* n = &T->n[node];
    if (t >= n->first) {
      qd = 0;
      if ((t - n->first) >= h->min_proc) {
        if ((n->second - (t + p)) >= h->min_proc) {
          int nx = ht_alloc(h, t + p, n->second);
          it_insert(T, nx);
          n = &T->n[node];
        }
        n->second = t;
      } else {
        if ((n->second - (t + p)) >= h->min_proc) { n->first = t + p; n->key = n->first; }
        else ht_release(h, it_remove(T, node));
      }
    } else {
      qd = n->first - t;
      if ((n->second - (n->first + p)) >= h->min_proc) { n->first = n->first + p; n->key = n->first; }
      else ht_release(h, it_remove(T, node));
    }
  }
  mg1_update(&h->m, t, p, qd);
  h->util_cycles += p;                            /* updateQueueUtilizationCounters */
  if (t + qd + p > h->last_req) h->last_req = t + qd + p;
  h->total_req++;
  return qd;
}

/* ======================================================================== */
/* NoC: NetworkModel + emesh_hop_counter + emesh_hop_by_hop                  */
/* ======================================================================== */
enum { P_SELF = 0, P_LEFT, P_RIGHT, P_DOWN, P_UP, NPORTS };   /* network_model_emesh_hop_by_hop.h:41-48 */

/* the model-specific parameter of oracle_qmodel_create for the router queues */
static uint32_t qm_aux_of(const gg_config* c, uint32_t type)
{
  return type == GG_QM_BASIC ? c->basic_moving_avg : c->history_list_no_interleaving;
}
static uint32_t qm_aux(const gg_config* c) { return qm_aux_of(c, c->queue_model_type); }

struct oracle_noc {
  gg_config cfg;
  uint32_t n, w, h, id_bits;
  oracle_htree** inj;      /* [tile]            _injection_router queue (1 port)   */
  oracle_htree** q;        /* [tile][NPORTS]    _mesh_router output-port queues     */
  uint64_t* c;             /* [tile][GG_NUM_NET_COUNTERS]                           */
};

oracle_noc* oracle_noc_create(const gg_config* cfg)
{
  oracle_noc* on = (oracle_noc*)calloc(1, sizeof(*on));
  on->cfg = *cfg;
  on->n = cfg->num_tiles;
  on->w = (uint32_t)floor(sqrt((double)cfg->num_tiles));        /* hop_counter.cc:18-19 */
  on->h = (uint32_t)ceil(1.0 * cfg->num_tiles / on->w);
  on->id_bits = (uint32_t)ceil_log2(cfg->num_tiles);            /* config.cc:149-152 */
  on->c = (uint64_t*)calloc((size_t)on->n * GG_NUM_NET_COUNTERS, sizeof(uint64_t));
  if (cfg->net_model == GG_NET_EMESH_HOP_BY_HOP && cfg->queue_model_enabled) {
    on->inj = (oracle_htree**)calloc(on->n, sizeof(void*));
    on->q = (oracle_htree**)calloc((size_t)on->n * NPORTS, sizeof(void*));
    for (uint32_t i = 0; i < on->n; ++i) {
      on->inj[i] = oracle_qmodel_create(cfg->queue_model_type, qm_aux(cfg), 1, (int)cfg->max_list_size, (int)cfg->analytical_enabled);
      for (int p = 0; p < NPORTS; ++p)       /* QueueModel::create(type, 1) (router_model.cc:23-27) */
        on->q[(size_t)i * NPORTS + p] = oracle_qmodel_create(cfg->queue_model_type, qm_aux(cfg), 1, (int)cfg->max_list_size,
                                                           (int)cfg->analytical_enabled);
    }
  }
  return on;
}

void oracle_noc_destroy(oracle_noc* on)
{
  if (!on) return;
  if (on->inj) {
    for (uint32_t i = 0; i < on->n; ++i) {
      oracle_htree_destroy(on->inj[i]);
      for (int p = 0; p < NPORTS; ++p) oracle_htree_destroy(on->q[(size_t)i * NPORTS + p]);
    }
    free(on->inj); free(on->q);
  }
  free(on->c); free(on);
}

void oracle_noc_counters(const oracle_noc* on, uint64_t* out)
{
  memcpy(out, on->c, sizeof(uint64_t) * on->n * GG_NUM_NET_COUNTERS);
  if (on->q) {
    for (uint32_t i = 0; i < on->n; ++i) {
      uint64_t a = 0;
      for (int p = 0; p < NPORTS; ++p) a += on->q[(size_t)i * NPORTS + p]->analytical_requests;
      out[(size_t)i * GG_NUM_NET_COUNTERS + GG_NC_ANALYTICAL_REQUESTS] = a;
      for (int p = 0; p < 5; ++p) {                /* mesh output ports: queue_model.cc:49-55 */
        out[(size_t)i * GG_NUM_NET_COUNTERS + GG_NC_PORT_UTILIZED_CYCLES + p] = on->q[(size_t)i * NPORTS + p]->util_cycles;
        out[(size_t)i * GG_NUM_NET_COUNTERS + GG_NC_PORT_LAST_CYCLES + p] = on->q[(size_t)i * NPORTS + p]->last_req;
      }
    }
  }
}

/* NetworkModel::computeNumFlits (network_model.cc:202-212) */
static uint64_t n_flits(const oracle_noc* on, uint32_t bits)
{
  uint32_t fw = on->cfg.flit_width;
  return (bits % fw == 0) ? bits / fw : bits / fw + 1;
}

static uint64_t* ncnt(oracle_noc* on, uint32_t tile) { return on->c + (size_t)tile * GG_NUM_NET_COUNTERS; }

/* updateSendCounters (network_model.cc:228-251) */
static void n_send_counters(oracle_noc* on, uint32_t src, uint32_t bits)
{
  uint64_t* c = ncnt(on, src);
  c[GG_NC_PACKETS_SENT]++; c[GG_NC_FLITS_SENT] += n_flits(on, bits); c[GG_NC_BITS_SENT] += bits;
}

/* __processReceivedPacket -> processReceivedPacket + updateReceiveCounters (network_model.cc:118-150,253-272) */
static void n_receive(oracle_noc* on, uint32_t dst, uint32_t bits, uint64_t* t, uint64_t* zl, uint64_t cont)
{
  uint64_t nf = n_flits(on, bits);
  uint64_t ser = lat_to_ps(nf, on->cfg.frequency_ghz);
  *t += ser; *zl += ser;
  uint64_t* c = ncnt(on, dst);
  c[GG_NC_PACKETS_RECEIVED]++; c[GG_NC_FLITS_RECEIVED] += nf; c[GG_NC_BITS_RECEIVED] += bits;
  c[GG_NC_TOTAL_LATENCY_PS] += *zl + cont;
  c[GG_NC_TOTAL_CONTENTION_PS] += cont;
}

/* binary min-heap of (time_ps, packet id) mesh-hop events */
typedef struct { uint64_t t; uint64_t id; } n_ev;
typedef struct { n_ev* a; uint64_t n, cap; } n_heap;
static int ev_lt(n_ev x, n_ev y) { return x.t < y.t || (x.t == y.t && x.id < y.id); }
static void heap_push(n_heap* h, n_ev e)
{
  if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 1024; h->a = (n_ev*)realloc(h->a, sizeof(n_ev) * h->cap); }
  uint64_t i = h->n++;
  while (i > 0) { uint64_t p = (i - 1) / 2; if (!ev_lt(e, h->a[p])) break; h->a[i] = h->a[p]; i = p; }
  h->a[i] = e;
}
static n_ev heap_pop(n_heap* h)
{
  n_ev top = h->a[0], last = h->a[--h->n];
  uint64_t i = 0;
  for (;;) {
    uint64_t l = 2 * i + 1, r = l + 1, m = i;
    n_ev cand = last;
    if (l < h->n && ev_lt(h->a[l], cand)) { m = l; cand = h->a[l]; }
    if (r < h->n && ev_lt(h->a[r], cand)) { m = r; }
    if (m == i) break;
    h->a[i] = h->a[m]; i = m;
  }
  if (h->n) h->a[i] = last;
  return top;
}

static int cmp_inj(const void* x, const void* y)
{
  const n_ev* a = (const n_ev*)x; const n_ev* b = (const n_ev*)y;
  return ev_lt(*a, *b) ? -1 : (ev_lt(*b, *a) ? 1 : 0);
}

static void noc_hbh_walk(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst, const uint32_t* len,
                         uint32_t* cur, uint64_t* t, uint64_t* zl, uint64_t* ct, const uint8_t* inj,
                         const uint32_t* shard, uint8_t* held);

/*
 * Route a batch.  emesh_hop_counter: one closed-form hop per packet
 * (network_model_emesh_hop_counter.cc:143-157).  emesh_hop_by_hop: the
 * canonical discrete-event order: the injection port of
 * every tile serves its packets in (send time, packet index) order, then every
 * mesh router output port serves the packets that reach it in (arrival time,
 * packet index) order — exactly what a single global event queue keyed
 * (time_ps, packet index) produces.
 */
int oracle_noc_route(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst,
                     const uint32_t* len, const uint64_t* time_ps,
                     uint64_t* arrival, uint64_t* zero_load, uint64_t* contention)
{
  const double f = on->cfg.frequency_ghz;
  for (uint64_t k = 0; k < n; ++k)
    if (src[k] >= on->n || dst[k] >= on->n) return GG_ERR_INVALID;

  if (on->cfg.net_model == GG_NET_MAGIC) {
    /* network_model_magic.cc:5-21: _flit_width = -1 (computeNumFlits -> 0 flits), one hop of 1 cycle */
    for (uint64_t k = 0; k < n; ++k) {
      uint64_t t = time_ps[k], zl = 0;
      if (src[k] != dst[k]) {
        uint64_t* cs = ncnt(on, src[k]);
        cs[GG_NC_PACKETS_SENT]++; cs[GG_NC_BITS_SENT] += len[k];
        uint64_t l1 = lat_to_ps(1, f);
        t += l1; zl += l1;
        uint64_t* cr = ncnt(on, dst[k]);
        cr[GG_NC_PACKETS_RECEIVED]++; cr[GG_NC_BITS_RECEIVED] += len[k];
        cr[GG_NC_TOTAL_LATENCY_PS] += zl;
      }
      arrival[k] = t; zero_load[k] = zl; contention[k] = 0;
    }
    return 0;
  }

  if (on->cfg.net_model == GG_NET_EMESH_HOP_COUNTER) {
    const uint64_t hop_latency = (uint64_t)on->cfg.router_delay + on->cfg.link_delay;  /* :81 */
    for (uint64_t k = 0; k < n; ++k) {
      uint64_t t = time_ps[k], zl = 0;
      if (src[k] != dst[k]) {                           /* processCornerCases (network_model.cc:413-424) */
        n_send_counters(on, src[k], len[k]);
        int sx = (int)(src[k] % on->w), sy = (int)(src[k] / on->w);
        int dx = (int)(dst[k] % on->w), dy = (int)(dst[k] / on->w);
        uint64_t hops = (uint64_t)(abs(sx - dx) + abs(sy - dy));
        uint64_t lat = lat_to_ps(hops * hop_latency, f);
        t += lat; zl += lat;                            /* Hop ctor (network_model.cc:556-563) */
        uint64_t nf = n_flits(on, len[k]);              /* updateEventCounters (:120-127) */
        uint64_t* c = ncnt(on, src[k]);
        c[GG_NC_BUFFER_WRITES] += nf * hops; c[GG_NC_BUFFER_READS] += nf * hops;
        c[GG_NC_SWITCH_ALLOC] += hops; c[GG_NC_CROSSBAR] += nf * hops; c[GG_NC_LINK_TRAVERSALS] += nf * hops;
        n_receive(on, dst[k], len[k], &t, &zl, 0);
      }
      arrival[k] = t; zero_load[k] = zl; contention[k] = 0;
    }
    return 0;
  }

  if (on->cfg.net_model != GG_NET_EMESH_HOP_BY_HOP) return GG_ERR_UNSUPPORTED;
  if (on->n != on->w * on->h) return GG_ERR_UNSUPPORTED;     /* hop_by_hop.cc:55-59 */
  uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  uint8_t* inj = (uint8_t*)malloc(n ? n : 1);
  for (uint64_t k = 0; k < n; ++k) {
    arrival[k] = time_ps[k]; zero_load[k] = 0; contention[k] = 0; cur[k] = src[k]; inj[k] = 1;
  }
  noc_hbh_walk(on, n, src, dst, len, cur, arrival, zero_load, contention, inj, NULL, NULL);
  free(cur); free(inj);
  return 0;
}

/*
 * emesh_hop_by_hop with broadcast packets (dst == GG_BROADCAST): the broadcast
 * tree of NetworkModelEMeshHopByHop::routePacket (hop_by_hop.cc:163-221).  A
 * broadcast event at router c = (cx, cy) of a packet sent by s = (sx, sy)
 * forks to UP if cy >= sy, DOWN if cy <= sy, and in the sender's row RIGHT if
 * cx >= sx, LEFT if cx <= sx — each only when that neighbour exists
 * (computeTileID, :274-280) — plus SELF (RECEIVE_TILE at c).  Every listed
 * link adds its delay (the max over equal link delays is link_delay, :185-205)
 * and RouterModel::processPacket(pkt, list) (router_model.cc:71-108) asks
 * every listed output-port queue and keeps the largest delay; its contention
 * counters add that max to each listed port (:135-143), the event counters
 * add one crossbar traversal of list size (:120-127).  Order: injection ports
 * first as in oracle_noc_route, then one global heap of (time, packet index)
 * events, each carrying its copy's zero-load / contention sums.  Unicast
 * packets take the XY hops of noc_hbh_walk.  Deliveries of the b-th broadcast
 * of the batch go to b_*[b * tiles + tile].
 */
typedef struct { uint64_t t, zl, ct, id; uint32_t at; } n_tev;
typedef struct { n_tev* a; uint64_t n, cap; } n_theap;
static int tev_lt(const n_tev* x, const n_tev* y) { return x->t < y->t || (x->t == y->t && x->id < y->id); }
static void theap_push(n_theap* h, n_tev e)
{
  if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 1024; h->a = (n_tev*)realloc(h->a, sizeof(n_tev) * h->cap); }
  uint64_t i = h->n++;
  while (i > 0) { uint64_t p = (i - 1) / 2; if (!tev_lt(&e, &h->a[p])) break; h->a[i] = h->a[p]; i = p; }
  h->a[i] = e;
}
static n_tev theap_pop(n_theap* h)
{
  n_tev top = h->a[0], last = h->a[--h->n];
  uint64_t i = 0;
  for (;;) {
    uint64_t l = 2 * i + 1, r = l + 1, m = i;
    const n_tev* cand = &last;
    if (l < h->n && tev_lt(&h->a[l], cand)) { m = l; cand = &h->a[l]; }
    if (r < h->n && tev_lt(&h->a[r], cand)) { m = r; }
    if (m == i) break;
    h->a[i] = h->a[m]; i = m;
  }
  if (h->n) h->a[i] = last;
  return top;
}

int oracle_noc_route_tree(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst,
                          const uint32_t* len, const uint64_t* time_ps,
                          uint64_t* arrival, uint64_t* zero_load, uint64_t* contention,
                          uint64_t* b_arrival, uint64_t* b_zero_load, uint64_t* b_contention)
{
  if (on->cfg.net_model != GG_NET_EMESH_HOP_BY_HOP) return GG_ERR_UNSUPPORTED;
  if (on->n != on->w * on->h) return GG_ERR_UNSUPPORTED;
  for (uint64_t k = 0; k < n; ++k)
    if (src[k] >= on->n || (dst[k] >= on->n && dst[k] != GG_BROADCAST)) return GG_ERR_INVALID;
  const double f = on->cfg.frequency_ghz;
  const int qm = on->cfg.queue_model_enabled != 0;
  const int W = (int)on->w, H = (int)on->h;
  uint64_t* bidx = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  uint64_t nb = 0;
  for (uint64_t k = 0; k < n; ++k) bidx[k] = dst[k] == GG_BROADCAST ? nb++ : ~0ull;
  n_theap heap = { 0, 0, 0 };
  /* 1. injection ports (SEND_TILE, :151-159) in (time, index) order per source */
  {
    uint64_t* cnt = (uint64_t*)calloc(on->n + 1, sizeof(uint64_t));
    for (uint64_t k = 0; k < n; ++k) {
      if (src[k] == dst[k]) { arrival[k] = time_ps[k]; zero_load[k] = 0; contention[k] = 0; continue; }
      cnt[src[k] + 1]++;
    }
    for (uint32_t s = 0; s < on->n; ++s) cnt[s + 1] += cnt[s];
    n_ev* by = (n_ev*)malloc(sizeof(n_ev) * (cnt[on->n] ? cnt[on->n] : 1));
    uint64_t* pos = (uint64_t*)malloc(sizeof(uint64_t) * (on->n + 1));
    memcpy(pos, cnt, sizeof(uint64_t) * (on->n + 1));
    for (uint64_t k = 0; k < n; ++k)
      if (src[k] != dst[k]) { n_ev e = { time_ps[k], k }; by[pos[src[k]]++] = e; }
    for (uint32_t s = 0; s < on->n; ++s) {
      qsort(by + cnt[s], cnt[s + 1] - cnt[s], sizeof(n_ev), cmp_inj);
      for (uint64_t i = cnt[s]; i < cnt[s + 1]; ++i) {
        uint64_t k = by[i].id;
        uint64_t nf = n_flits(on, len[k]);
        n_send_counters(on, s, len[k]);
        if (dst[k] == GG_BROADCAST) {                      /* updateSendCounters (network_model.cc:244-250) */
          uint64_t* cs = ncnt(on, s);
          cs[GG_NC_PACKETS_BROADCASTED]++; cs[GG_NC_FLITS_BROADCASTED] += nf; cs[GG_NC_BITS_BROADCASTED] += len[k];
        }
        uint64_t qd = qm ? oracle_htree_delay(on->inj[s], time_to_cycles(time_ps[k], f), nf) : 0;
        uint64_t cps = lat_to_ps(qd, f);
        n_tev e = { time_ps[k] + lat_to_ps(0, f) + cps, 0, cps, k, s };
        theap_push(&heap, e);
      }
    }
    free(cnt); free(by); free(pos);
  }
  /* 2. mesh routers in global (time, index) order */
  while (heap.n) {
    n_tev e = theap_pop(&heap);
    uint64_t k = e.id;
    uint32_t c = e.at;
    int cx = (int)(c % on->w), cy = (int)(c / on->w);
    int ports[5], np = 0;
    uint32_t nxt[5];
    if (dst[k] != GG_BROADCAST) {
      int dx = (int)(dst[k] % on->w), dy = (int)(dst[k] / on->w);
      if (cx > dx)      { ports[0] = P_LEFT;  nxt[0] = c - 1; }
      else if (cx < dx) { ports[0] = P_RIGHT; nxt[0] = c + 1; }
      else if (cy > dy) { ports[0] = P_DOWN;  nxt[0] = c - on->w; }
      else if (cy < dy) { ports[0] = P_UP;    nxt[0] = c + on->w; }
      else              { ports[0] = P_SELF;  nxt[0] = c; }
      np = 1;
    } else {
      int sx = (int)(src[k] % on->w), sy = (int)(src[k] / on->w);
      if (cy >= sy && cy + 1 < H) { ports[np] = P_UP;    nxt[np++] = c + on->w; }
      if (cy <= sy && cy - 1 >= 0) { ports[np] = P_DOWN;  nxt[np++] = c - on->w; }
      if (cy == sy) {
        if (cx >= sx && cx + 1 < W) { ports[np] = P_RIGHT; nxt[np++] = c + 1; }
        if (cx <= sx && cx - 1 >= 0) { ports[np] = P_LEFT;  nxt[np++] = c - 1; }
      }
      ports[np] = P_SELF; nxt[np++] = c;
    }
    uint64_t nf = n_flits(on, len[k]);
    uint64_t zlc = (uint64_t)on->cfg.router_delay + on->cfg.link_delay, qd = 0;
    uint64_t* cc = ncnt(on, c);
    if (qm) {
      for (int i = 0; i < np; ++i) {
        uint64_t d = oracle_htree_delay(on->q[(size_t)c * NPORTS + ports[i]], time_to_cycles(e.t, f), nf);
        if (d > qd) qd = d;
      }
      cc[GG_NC_ROUTER_CONTENTION_CYCLES] += qd * (uint64_t)np; cc[GG_NC_ROUTER_PACKETS] += (uint64_t)np;
    }
    cc[GG_NC_BUFFER_WRITES] += nf; cc[GG_NC_BUFFER_READS] += nf; cc[GG_NC_SWITCH_ALLOC] += 1;
    if (np == 1) cc[GG_NC_CROSSBAR] += nf; else cc[GG_NC_CROSSBAR_MULTI + np - 2] += nf;
    cc[GG_NC_LINK_TRAVERSALS] += nf * (uint64_t)np;
    uint64_t zps = lat_to_ps(zlc, f), cps = lat_to_ps(qd, f);
    uint64_t t = e.t + zps + cps, zl = e.zl + zps, ct = e.ct + cps;
    for (int i = 0; i < np; ++i) {
      if (ports[i] == P_SELF) {
        uint64_t tt = t, zz = zl;
        n_receive(on, c, len[k], &tt, &zz, ct);
        if (dst[k] == GG_BROADCAST) {
          size_t o = (size_t)bidx[k] * on->n + c;
          b_arrival[o] = tt; b_zero_load[o] = zz; b_contention[o] = ct;
        } else {
          arrival[k] = tt; zero_load[k] = zz; contention[k] = ct;
        }
      } else {
        n_tev ne = { t, zl, ct, k, nxt[i] };
        theap_push(&heap, ne);
      }
    }
  }
  free(heap.a); free(bidx);
  return 0;
}

/*
 * emesh_hop_by_hop walk of a batch (hop_by_hop.cc:146-264) in the canonical
 * discrete-event order: the injection port of every tile serves its NEW
 * packets (inj[k] != 0) in (time, packet index) order (routePacket SEND_TILE,
 * :151-159), then every mesh router output port serves the packets that reach
 * it in (arrival time, packet index) order — what one global event queue keyed
 * (time_ps, packet index) produces.  Packet state in/out: cur (router tile),
 * t (time), zl, ct.  With a tile -> logical shard table `shard`, a packet whose
 * next router lies in another shard stops after the output port + link of its
 * current router (held[k] = 1, cur[k] = that next router): it continues there
 * after the quantum boundary.  Self packets (src == dst)
 * are left untouched (processCornerCases, network_model.cc:413-424).
 */
/* One hop of packet k at router cur[k] (hop_by_hop.cc:223-256): XY port
 * choice, RouterModel::processPacket (router_model.cc:71-108) through the
 * port's queue, ElectricalLinkModel (electrical_link_model.cc:31-45); at the
 * destination's SELF port the packet is received (network_model.cc:142-150). */
enum { HOP_MOVED = 0, HOP_DELIVERED, HOP_HELD };
static int hbh_hop(oracle_noc* on, uint64_t k, const uint32_t* dst, const uint32_t* len, uint32_t* cur,
                   uint64_t* t, uint64_t* zl, uint64_t* ct, const uint32_t* shard, uint8_t* held)
{
  const double f = on->cfg.frequency_ghz;
  const uint32_t c = cur[k];
  const int cx = (int)(c % on->w), cy = (int)(c / on->w);
  const int dx = (int)(dst[k] % on->w), dy = (int)(dst[k] / on->w);
  int port; uint32_t next;
  if (cx > dx)      { port = P_LEFT;  next = c - 1; }
  else if (cx < dx) { port = P_RIGHT; next = c + 1; }
  else if (cy > dy) { port = P_DOWN;  next = c - on->w; }
  else if (cy < dy) { port = P_UP;    next = c + on->w; }
  else              { port = P_SELF;  next = c; }
  const uint64_t nf = n_flits(on, len[k]);
  uint64_t zlc = on->cfg.router_delay, qd = 0;
  uint64_t* cc = ncnt(on, c);
  if (on->cfg.queue_model_enabled) {
    qd = oracle_htree_delay(on->q[(size_t)c * NPORTS + port], time_to_cycles(t[k], f), nf);
    cc[GG_NC_ROUTER_CONTENTION_CYCLES] += qd; cc[GG_NC_ROUTER_PACKETS]++;
  }
  cc[GG_NC_BUFFER_WRITES] += nf; cc[GG_NC_BUFFER_READS] += nf; cc[GG_NC_SWITCH_ALLOC] += 1; cc[GG_NC_CROSSBAR] += nf;
  zlc += on->cfg.link_delay;
  cc[GG_NC_LINK_TRAVERSALS] += nf;
  const uint64_t zps = lat_to_ps(zlc, f), cps = lat_to_ps(qd, f);
  t[k] += zps + cps; zl[k] += zps; ct[k] += cps;
  if (port == P_SELF) { n_receive(on, dst[k], len[k], &t[k], &zl[k], ct[k]); return HOP_DELIVERED; }
  cur[k] = next;
  if (shard && shard[next] != shard[c]) { held[k] = 1; return HOP_HELD; }   /* leaves the shard: held */
  return HOP_MOVED;
}

static void noc_hbh_walk(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst, const uint32_t* len,
                         uint32_t* cur, uint64_t* t, uint64_t* zl, uint64_t* ct, const uint8_t* inj,
                         const uint32_t* shard, uint8_t* held)
{
  const double f = on->cfg.frequency_ghz;
  const int qm = on->cfg.queue_model_enabled != 0;
  n_heap heap = { 0, 0, 0 };
  /* 1. injection ports of the new packets: stable grouping by source, (time, index) order */
  {
    uint64_t* cnt = (uint64_t*)calloc(on->n + 1, sizeof(uint64_t));
    uint64_t ninj = 0;
    for (uint64_t k = 0; k < n; ++k) if (inj[k] && src[k] != dst[k]) { cnt[src[k] + 1]++; ninj++; }
    for (uint32_t s = 0; s < on->n; ++s) cnt[s + 1] += cnt[s];
    n_ev* by = (n_ev*)malloc(sizeof(n_ev) * (ninj ? ninj : 1));
    uint64_t* pos = (uint64_t*)malloc(sizeof(uint64_t) * (on->n + 1));
    memcpy(pos, cnt, sizeof(uint64_t) * (on->n + 1));
    for (uint64_t k = 0; k < n; ++k) {
      if (src[k] == dst[k]) continue;                            /* self: zero time, no counters */
      if (inj[k]) { n_ev e = { t[k], k }; by[pos[src[k]]++] = e; }
      else { n_ev e = { t[k], k }; heap_push(&heap, e); }          /* held packet resuming at cur[k] */
    }
    for (uint32_t s = 0; s < on->n; ++s) {
      uint64_t b = cnt[s], e = cnt[s + 1];
      qsort(by + b, e - b, sizeof(n_ev), cmp_inj);
      for (uint64_t i = b; i < e; ++i) {
        uint64_t k = by[i].id;
        n_send_counters(on, src[k], len[k]);
        uint64_t qd = 0;
        if (qm) qd = oracle_htree_delay(on->inj[s], time_to_cycles(t[k], f), n_flits(on, len[k]));
        uint64_t cps = lat_to_ps(qd, f);
        t[k] += lat_to_ps(0, f) + cps; ct[k] += cps;
        n_ev ev = { t[k], k };
        heap_push(&heap, ev);
      }
    }
    free(cnt); free(by); free(pos);
  }
  /* 2. mesh hops in global (time, index) order (hop_by_hop.cc:223-256) */
  while (heap.n) {
    n_ev ev = heap_pop(&heap);
    const uint64_t k = ev.id;
    if (hbh_hop(on, k, dst, len, cur, t, zl, ct, shard, held) == HOP_MOVED) {
      n_ev ne = { t[k], k };
      heap_push(&heap, ne);
    }
  }
  free(heap.a);
}

/* The same walk, stage by stage on `threads` OpenMP threads (the tile-parallel
 * CPU baseline, oracle_coh_set_threads).  A port's requests depend only on the
 * ports before it on the packets' XY routes, and its order is (arrival time,
 * packet index) whatever else runs: so the injection ports (per source), then
 * the X hops row by row (each direction swept in its direction of travel,
 * each position's batch in (time, index) order), then the Y hops column by
 * column, then the SELF ports (per destination) see exactly the requests, in
 * exactly the order, of the global event queue above — the GPU's stage
 * decomposition.  Rows / columns / tiles run in parallel: each
 * touches only its own routers' queues and counters. */
static void hbh_sweep(oracle_noc* on, uint64_t m, uint64_t* ids, uint32_t npos, int stage, int dir,
                      const uint32_t* dst, const uint32_t* len, uint32_t* cur, uint64_t* t, uint64_t* zl,
                      uint64_t* ct, const uint32_t* shard, uint8_t* held, n_ev* tmp, uint64_t* nxt, uint64_t* head)
{
  /* per position a list of the packets there (row / column-local indices into ids) */
  for (uint32_t p = 0; p < npos; ++p) head[p] = ~0ull;
  const uint32_t W = on->w;
  for (uint64_t i = 0; i < m; ++i) {
    const uint32_t c = cur[ids[i]], p = stage == 0 ? c % W : c / W;
    nxt[i] = head[p]; head[p] = i;
  }
  for (uint32_t s = 0; s < npos; ++s) {
    const uint32_t p = dir > 0 ? s : npos - 1 - s;
    uint64_t nb = 0;
    for (uint64_t i = head[p]; i != ~0ull; i = nxt[i]) { n_ev e = { t[ids[i]], i }; tmp[nb++] = e; }
    if (!nb) continue;
    for (uint64_t j = 0; j < nb; ++j) tmp[j].id = ids[tmp[j].id] << 20 | tmp[j].id;   /* order by packet index */
    qsort(tmp, nb, sizeof(n_ev), cmp_inj);
    for (uint64_t j = 0; j < nb; ++j) {
      const uint64_t i = tmp[j].id & ((1u << 20) - 1), k = tmp[j].id >> 20;
      if (hbh_hop(on, k, dst, len, cur, t, zl, ct, shard, held) != HOP_MOVED) continue;
      const uint32_t c = cur[k], dx = dst[k] % W, dy = dst[k] / W;
      if (stage == 0 ? c % W == dx : c / W == dy) continue;          /* this stage is over for k */
      const uint32_t q = stage == 0 ? c % W : c / W;                 /* the next position, later in the sweep */
      nxt[i] = head[q]; head[q] = i;
    }
  }
}

static void noc_hbh_walk_par(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst, const uint32_t* len,
                             uint32_t* cur, uint64_t* t, uint64_t* zl, uint64_t* ct, const uint8_t* inj,
                             const uint32_t* shard, uint8_t* held, int threads)
{
  const double f = on->cfg.frequency_ghz;
  const int qm = on->cfg.queue_model_enabled != 0;
  const uint32_t W = on->w, H = on->h, T = on->n;
  if (n >= (1ull << 20)) { noc_hbh_walk(on, n, src, dst, len, cur, t, zl, ct, inj, shard, held); return; }
  uint32_t* key = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  uint64_t* cnt = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)T + 1));
  uint64_t* ids = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  /* group the packets k with key[k] < nk by key (stable): ids[cnt[g] .. cnt[g+1]) */
#define GROUP(nk)                                                                  \
  do {                                                                             \
    memset(cnt, 0, sizeof(uint64_t) * ((size_t)(nk) + 1));                         \
    for (uint64_t k = 0; k < n; ++k) if (key[k] < (nk)) cnt[key[k] + 1]++;         \
    for (uint32_t g = 0; g < (nk); ++g) cnt[g + 1] += cnt[g];                      \
    uint64_t* pos_ = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)(nk) + 1));     \
    memcpy(pos_, cnt, sizeof(uint64_t) * ((size_t)(nk) + 1));                      \
    for (uint64_t k = 0; k < n; ++k) if (key[k] < (nk)) ids[pos_[key[k]]++] = k;   \
    free(pos_);                                                                    \
  } while (0)
  /* 1. injection ports, per source */
  for (uint64_t k = 0; k < n; ++k) key[k] = (inj[k] && src[k] != dst[k]) ? src[k] : ~0u;
  GROUP(T);
#pragma omp parallel num_threads(threads)
  {
    n_ev* by = (n_ev*)malloc(sizeof(n_ev) * (n ? n : 1));
#pragma omp for schedule(dynamic, 16)
    for (uint32_t s = 0; s < T; ++s) {
      const uint64_t b = cnt[s], e = cnt[s + 1];
      for (uint64_t i = b; i < e; ++i) { n_ev x = { t[ids[i]], ids[i] }; by[i - b] = x; }
      qsort(by, e - b, sizeof(n_ev), cmp_inj);
      for (uint64_t i = 0; i < e - b; ++i) {
        const uint64_t k = by[i].id;
        n_send_counters(on, src[k], len[k]);
        uint64_t qd = 0;
        if (qm) qd = oracle_htree_delay(on->inj[s], time_to_cycles(t[k], f), n_flits(on, len[k]));
        const uint64_t cps = lat_to_ps(qd, f);
        t[k] += lat_to_ps(0, f) + cps; ct[k] += cps;
      }
    }
    free(by);
  }
  /* 2-3. X hops per row, Y hops per column */
  for (int stage = 0; stage < 2; ++stage) {
    const uint32_t nlines = stage == 0 ? H : W, npos = stage == 0 ? W : H;
    for (uint64_t k = 0; k < n; ++k) {
      key[k] = ~0u;
      if (src[k] == dst[k] || held[k]) continue;
      const uint32_t c = cur[k];
      if (stage == 0 && c % W != dst[k] % W) key[k] = c / W;
      if (stage == 1 && c % W == dst[k] % W && c / W != dst[k] / W) key[k] = c % W;
    }
    GROUP(nlines);
#pragma omp parallel num_threads(threads)
    {
      n_ev* tmp = (n_ev*)malloc(sizeof(n_ev) * (n ? n : 1));
      uint64_t* nxt = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
      uint64_t* head = (uint64_t*)malloc(sizeof(uint64_t) * npos);
      uint64_t* sub = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
#pragma omp for schedule(dynamic, 1)
      for (uint32_t ln = 0; ln < nlines; ++ln) {
        /* the line's packets by direction (before either sweep moves them): RIGHT / UP, then LEFT / DOWN */
        const uint64_t b = cnt[ln], e = cnt[ln + 1];
        uint64_t m = 0, r = e - b;
        for (uint64_t i = b; i < e; ++i) {
          const uint64_t k = ids[i];
          const uint32_t c = cur[k];
          if (stage == 0 ? dst[k] % W > c % W : dst[k] / W > c / W) sub[m++] = k;
          else sub[--r] = k;
        }
        if (m) hbh_sweep(on, m, sub, npos, stage, 1, dst, len, cur, t, zl, ct, shard, held, tmp, nxt, head);
        if (e - b > m) hbh_sweep(on, e - b - m, sub + m, npos, stage, -1, dst, len, cur, t, zl, ct, shard, held, tmp, nxt, head);
      }
      free(tmp); free(nxt); free(head); free(sub);
    }
  }
  /* 4. SELF ports, per destination */
  for (uint64_t k = 0; k < n; ++k) key[k] = (src[k] != dst[k] && !held[k] && cur[k] == dst[k]) ? dst[k] : ~0u;
  GROUP(T);
#pragma omp parallel num_threads(threads)
  {
    n_ev* by = (n_ev*)malloc(sizeof(n_ev) * (n ? n : 1));
#pragma omp for schedule(dynamic, 16)
    for (uint32_t d = 0; d < T; ++d) {
      const uint64_t b = cnt[d], e = cnt[d + 1];
      for (uint64_t i = b; i < e; ++i) { n_ev x = { t[ids[i]], ids[i] }; by[i - b] = x; }
      qsort(by, e - b, sizeof(n_ev), cmp_inj);
      for (uint64_t i = 0; i < e - b; ++i) hbh_hop(on, by[i].id, dst, len, cur, t, zl, ct, shard, held);
    }
    free(by);
  }
#undef GROUP
  free(key); free(cnt); free(ids);
}
#include "gg_coherent.inc"
