// gg_capi.hip — the extern "C" boundary (include/graphite_gpu.h): context
// lifetime, geometry, dispatch, error reporting and HIP-event kernel timing.
#include "gg_internal.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>

namespace {
thread_local std::string g_last_error;

__global__ void k_gen_uniform(uint64_t* addr, uint32_t* meta, uint32_t tile_begin, uint32_t tiles,
                              uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)tiles * per_tile) return;
  const uint32_t t = tile_begin + (uint32_t)(i / per_tile);
  const uint64_t k = first + i % per_tile;
  uint64_t z = (0x9E3779B97F4A7C15ull ^ (uint64_t)t) + (k + 1) * 0x9E3779B97F4A7C15ull;   // SplitMix64
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  addr[i] = ((uint64_t)t << base_shift) + ((z & ((1ull << lines_log2) - 1)) << 6);
  meta[i] = (((z >> 32) % 3) == 0) ? GG_META_WRITE : 0u;
}

// configs[2..4] hotspot generator (the same bit recipe as
// oracle_gen_hotspot, the checker)
__global__ void k_gen_hotspot(uint64_t* addr, uint32_t* meta, uint32_t tile_begin, uint32_t tiles, uint64_t per_tile,
                              uint64_t first, uint32_t lines_log2, uint32_t base_shift, uint32_t hot_lines,
                              uint32_t hot_frac256)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)tiles * per_tile) return;
  const uint32_t t = tile_begin + (uint32_t)(i / per_tile);
  const uint64_t k = first + i % per_tile;
  uint64_t z = (0x9E3779B97F4A7C15ull ^ (uint64_t)t) + (k + 1) * 0x9E3779B97F4A7C15ull;   // SplitMix64
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const bool hot = hot_lines && (((z >> 40) & 0xFF) < hot_frac256);
  addr[i] = hot ? (1ull << 44) + ((z & 0xFFFFFFFFull) % hot_lines) * 64ull
                : ((uint64_t)t << base_shift) + ((z & ((1ull << lines_log2) - 1)) << 6);
  const uint32_t gap = (uint32_t)__builtin_ctz((uint32_t)(((z >> 48) & 0xFF) | 0x100)) +
                       (uint32_t)__builtin_ctz((uint32_t)(((z >> 56) & 0xFF) | 0x100));
  meta[i] = ((((z >> 32) & 0xFF) % 3) == 0 ? GG_META_WRITE : 0u) | (gap << 1);
}

// configs[4] coherent stress generator (the same bit
// recipe as oracle_gen_stress, the checker): WRITE p = 1/2; with p =
// pool_frac256 / 256 a line of the shared pool [0, pool_lines) at byte 2^45,
// else a private line.  Tiles fall into max(1, T/64) groups by a 32-bit hash
// of the tile id; pool line L is shared by group L mod groups, and a tile's
// pool accesses pick among its group's lines, so every pool line has ~64
// sharers spread over the mesh.
__host__ __device__ inline uint32_t stress_group(uint32_t t, uint32_t groups)
{
  uint32_t x = t + 0x9E3779B9u;                      // lowbias32
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x % groups;
}
__global__ void k_gen_stress(uint64_t* addr, uint32_t* meta, uint32_t tile_begin, uint32_t tiles, uint64_t per_tile,
                             uint64_t first, uint32_t lines_log2, uint32_t base_shift, uint32_t num_tiles,
                             uint32_t pool_lines, uint32_t pool_frac256)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)tiles * per_tile) return;
  const uint32_t t = tile_begin + (uint32_t)(i / per_tile);
  const uint64_t k = first + i % per_tile;
  uint64_t z = (0x9E3779B97F4A7C15ull ^ (uint64_t)t) + (k + 1) * 0x9E3779B97F4A7C15ull;   // SplitMix64
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const uint32_t groups = num_tiles >= 128 ? num_tiles / 64 : 1;
  const uint32_t per_group = pool_lines / groups ? pool_lines / groups : 1;
  const bool pool = pool_lines && (((z >> 40) & 0xFF) < pool_frac256);
  addr[i] = pool ? (1ull << 45) + (uint64_t)(stress_group(t, groups) + groups * ((uint32_t)(z & 0xFFFFFFFFull) % per_group)) * 64ull
                 : ((uint64_t)t << base_shift) + ((z & ((1ull << lines_log2) - 1)) << 6);
  const uint32_t gap = (uint32_t)__builtin_ctz((uint32_t)(((z >> 48) & 0xFF) | 0x100)) +
                       (uint32_t)__builtin_ctz((uint32_t)(((z >> 56) & 0xFF) | 0x100));
  meta[i] = (uint32_t)((z >> 32) & 1u) * GG_META_WRITE | (gap << 1);
}

int floor_log2(uint64_t n) { int p = -1; while (n) { n >>= 1; ++p; } return p; }
bool is_pow2(uint64_t n) { return n && !(n & (n - 1)); }
}  // namespace

gg_status gg_fail(gg_status code, const char* fmt, ...)
{
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

gg_status gg_hip_check(hipError_t e, const char* what)
{
  return gg_fail(GG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

void gg_timer_begin(gg_ctx* ctx, const char* name, hipStream_t s)
{
  if (!ctx->timing) return;
  for (gg_timer& t : ctx->timers)
    if (t.name == name) { hipEventRecord(t.start, s); t.valid = false; return; }
  gg_timer t;
  t.name = name;
  hipEventCreate(&t.start);
  hipEventCreate(&t.stop);
  hipEventRecord(t.start, s);
  ctx->timers.push_back(t);
}

void gg_timer_end(gg_ctx* ctx, const char* name, hipStream_t s)
{
  if (!ctx->timing) return;
  for (gg_timer& t : ctx->timers)
    if (t.name == name) { hipEventRecord(t.stop, s); t.valid = true; return; }
}

extern "C" {

int gg_abi_version(void) { return GG_ABI_VERSION; }
const char* gg_last_error(void) { return g_last_error.c_str(); }

void gg_config_default(gg_config* c, uint32_t num_tiles)
{
  memset(c, 0, sizeof(*c));
  c->num_tiles = num_tiles;
  c->line_size = 64;
  c->l1d_size_kb = 32; c->l1d_assoc = 4; c->l1d_policy = GG_POLICY_LRU;
  c->l2_size_kb = 512; c->l2_assoc = 8; c->l2_policy = GG_POLICY_LRU;
  c->net_model = GG_NET_EMESH_HOP_COUNTER;
  c->flit_width = 64;
  c->router_delay = 1;
  c->link_delay = 1;
  c->queue_model_enabled = 1;
  c->max_list_size = 100;
  c->analytical_enabled = 1;
  c->frequency_ghz = 1.0;
  c->device = 0;
  c->l1d_data_cycles = 1; c->l1d_tags_cycles = 1;       /* carbon_sim.cfg:219-228 */
  c->l2_data_cycles = 8; c->l2_tags_cycles = 3;         /* carbon_sim.cfg:230-239 */
  c->dir_assoc = 16; c->dir_total_entries = 0; c->dir_access_cycles = 0;   /* :253-258 ("auto") */
  c->dram_latency_ns = 100; c->dram_bandwidth = 5.0f; c->dram_queue_model_enabled = 1;  /* :265-273 */
  c->quantum_ns = 1000;                                 /* :97 */
  c->num_shards = 1;
}

gg_ctx* gg_create(const gg_config* cfg, gg_status* status)
{
  gg_status dummy;
  if (!status) status = &dummy;
  if (!cfg || cfg->num_tiles == 0) { *status = gg_fail(GG_ERR_INVALID, "config NULL or zero tiles"); return nullptr; }
  const gg_config& c = *cfg;
  if (!is_pow2(c.line_size)) { *status = gg_fail(GG_ERR_INVALID, "line size must be a power of two"); return nullptr; }
  const uint64_t l1_sets = (uint64_t)c.l1d_size_kb * 1024 / ((uint64_t)c.l1d_assoc * c.line_size);
  const uint64_t l2_sets = (uint64_t)c.l2_size_kb * 1024 / ((uint64_t)c.l2_assoc * c.line_size);
  if (!is_pow2(l1_sets) || !is_pow2(l2_sets)) {
    *status = gg_fail(GG_ERR_UNSUPPORTED, "set counts must be powers of two (cache_hash_fn.h masks the set index)");
    return nullptr;
  }
  if (l2_sets < l1_sets) {
    *status = gg_fail(GG_ERR_UNSUPPORTED, "private replay needs L2 sets >= L1-D sets (L2 sets nest in L1-D sets)");
    return nullptr;
  }
  if (l1_sets > 1024) { *status = gg_fail(GG_ERR_UNSUPPORTED, "more than 1024 L1-D sets"); return nullptr; }
  if (c.l1d_assoc > 8 || c.l2_assoc > 32) { *status = gg_fail(GG_ERR_UNSUPPORTED, "associativity beyond 8 (L1-D) / 32 (L2)"); return nullptr; }
  if (c.l1d_policy > GG_POLICY_ROUND_ROBIN || c.l2_policy > GG_POLICY_ROUND_ROBIN) {
    *status = gg_fail(GG_ERR_INVALID, "unknown replacement policy");
    return nullptr;
  }
  if (c.frequency_ghz <= 0) { *status = gg_fail(GG_ERR_INVALID, "frequency must be positive"); return nullptr; }

  hipError_t he = hipSetDevice(c.device);
  if (he != hipSuccess) { *status = gg_hip_check(he, "hipSetDevice"); return nullptr; }

  gg_ctx* ctx = new gg_ctx();
  ctx->cfg = c;
  ctx->device = c.device;
  if (hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, c.device) != hipSuccess || ctx->num_cus <= 0)
    ctx->num_cus = 256;
  ctx->replay_variant = (int)c.replay_kernel;
  gg_geom& g = ctx->g;
  g.tiles = c.num_tiles;
  g.log_line = floor_log2(c.line_size);
  g.u1 = (uint32_t)l1_sets;
  g.log_u1 = floor_log2(l1_sets);
  g.a1 = c.l1d_assoc;
  g.l2_sets = (uint32_t)l2_sets;
  g.log_l2 = floor_log2(l2_sets);
  g.s2 = (uint32_t)(l2_sets / l1_sets);
  g.a2 = c.l2_assoc;
  g.mw = (c.l2_assoc + 7) / 8;
  g.pol1 = c.l1d_policy;
  g.pol2 = c.l2_policy;
  g.units = (uint64_t)g.tiles * g.u1;
  // L2 tags are stored as (line >> log2(L2 sets)) in 32 bits, 2^32-1 = invalid
  const uint32_t lim_shift = 32 + g.log_l2 + g.log_line;
  g.addr_limit = (lim_shift >= 64) ? ~0ull : ((0xFFFFFFFFull << (g.log_l2 + g.log_line)));

  gg_status st = gg_cache_state_alloc(ctx);
  if (st == GG_OK) st = gg_noc_alloc(ctx);
  if (st == GG_OK) {
    he = hipMalloc((void**)&ctx->err_dev, 2 * sizeof(uint32_t));   // flags, first failing source line (coherent)
    if (he != hipSuccess) st = gg_hip_check(he, "hipMalloc(err)");
  }
  if (st == GG_OK) st = gg_reset(ctx);
  if (st != GG_OK) { gg_destroy(ctx); *status = st; return nullptr; }
  *status = GG_OK;
  return ctx;
}

void gg_destroy(gg_ctx* ctx)
{
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipDeviceSynchronize();
  gg_cache_state_free(ctx);
  gg_noc_free(ctx);
  gg_coh_free(ctx);
  gg_core_free(ctx);
  if (ctx->round && ctx->round_free) ctx->round_free(ctx->round);
  if (ctx->err_dev) hipFree(ctx->err_dev);
  for (gg_timer& t : ctx->timers) { hipEventDestroy(t.start); hipEventDestroy(t.stop); }
  delete ctx;
}

gg_status gg_reset(gg_ctx* ctx)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "ctx NULL");
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->last_stream;
  if (gg_status st = gg_cache_state_reset(ctx, s)) return st;
  if (gg_status st = gg_noc_reset(ctx, s)) return st;
  GG_HIP(hipMemsetAsync(ctx->err_dev, 0, 2 * sizeof(uint32_t), s));
  GG_HIP(hipStreamSynchronize(s));
  return GG_OK;
}

static gg_status check_device_errors(gg_ctx* ctx)
{
  uint32_t e = 0;
  GG_HIP(hipMemcpy(&e, ctx->err_dev, sizeof(e), hipMemcpyDeviceToHost));
  if (e & GG_DERR_BARRIER)
    return gg_fail(GG_ERR_UNSUPPORTED, "a BARRIER record (GG_META_BARRIER) in a private-cache trace: barriers are "
                   "released by gg_coherent_run only; the batch's results and counters are not valid");
  if (e & GG_DERR_RANGE) return gg_fail(GG_ERR_RANGE, "a trace address is beyond the compressed-tag range (%#llx)",
                                        (unsigned long long)ctx->g.addr_limit);
  if (e & GG_DERR_STATE) return gg_fail(GG_ERR_STATE, "cache state the reference would reject (LOG_ASSERT_ERROR)");
  if (e & GG_DERR_CAP) return gg_fail(GG_ERR_HIP, "a device-side capacity or hand-off bound was exceeded");
  return GG_OK;
}

gg_status gg_cache_access_batch(gg_ctx* ctx, const gg_trace* trace, uint32_t* result_dev,
                                uint64_t* evicted_dev, void* stream)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "ctx NULL");
  if (ctx->cfg.l1i_track_miss_types || ctx->cfg.l2_track_miss_types)
    return gg_fail(GG_ERR_UNSUPPORTED, "miss-type tracking is built for the coherent mode only");
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  return gg_cache_run_batch(ctx, trace, result_dev, evicted_dev, s);
}

gg_status gg_cache_get_counters(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  GG_HIP(hipMemcpy(out, ctx->cs.counters, sizeof(uint64_t) * ctx->g.tiles * 2 * GG_NUM_CACHE_COUNTERS,
                   hipMemcpyDeviceToHost));
  return check_device_errors(ctx);
}

gg_status gg_cache_get_line_info(gg_ctx* ctx, uint32_t tile, int level, uint64_t addr, gg_line_info* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  return gg_cache_quartet(ctx, 0, tile, level, addr, nullptr, out, nullptr, nullptr);
}

gg_status gg_cache_set_line_info(gg_ctx* ctx, uint32_t tile, int level, uint64_t addr, const gg_line_info* in)
{
  if (!ctx || !in) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  return gg_cache_quartet(ctx, 1, tile, level, addr, in, nullptr, nullptr, nullptr);
}

gg_status gg_cache_access_line(gg_ctx* ctx, uint32_t tile, int level, uint64_t addr, int is_store)
{
  if (!ctx) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  return gg_cache_quartet(ctx, is_store ? 3 : 2, tile, level, addr, nullptr, nullptr, nullptr, nullptr);
}

gg_status gg_cache_insert_line(gg_ctx* ctx, uint32_t tile, int level, uint64_t addr, const gg_line_info* in,
                               int* eviction, uint64_t* evicted_addr, gg_line_info* evicted_info)
{
  if (!ctx || !in || !eviction || !evicted_addr || !evicted_info) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  return gg_cache_quartet(ctx, 4, tile, level, addr, in, evicted_info, eviction, evicted_addr);
}

gg_status gg_noc_route_batch(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out, void* stream)
{
  if (!ctx || !pk || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  return gg_noc_run(ctx, pk, out, s);
}

gg_status gg_noc_route_tree(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out,
                            const gg_packet_out* bcast_out, uint64_t num_broadcasts, void* stream)
{
  if (!ctx || !pk || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  ctx->last_stream = s;
  return gg_noc_tree(ctx, pk, out, bcast_out, num_broadcasts, s);
}

gg_status gg_noc_get_counters(gg_ctx* ctx, uint64_t* out)
{
  if (!ctx || !out) return gg_fail(GG_ERR_INVALID, "NULL argument");
  hipSetDevice(ctx->device);
  GG_HIP(hipStreamSynchronize(ctx->last_stream));
  if (gg_status st = gg_noc_counters(ctx, out)) return st;
  return check_device_errors(ctx);
}

gg_status gg_queue_delay_batch(gg_ctx* ctx, uint64_t min_processing_time, const uint64_t* pkt_time,
                               const uint64_t* proc_time, uint64_t n, uint64_t* delay_out)
{
  if (!ctx || (n && (!pkt_time || !proc_time || !delay_out))) return gg_fail(GG_ERR_INVALID, "NULL argument");
  // every reference queue has min_processing_time >= 1 and processing times
  // >= 1 (router_model.cc:23-27, dram_perf_model.cc:48,92): the interval
  // representation of gg_dev.h relies on it
  if (min_processing_time == 0) return gg_fail(GG_ERR_UNSUPPORTED, "min_processing_time 0");
  hipSetDevice(ctx->device);
  GG_HIP(hipMemset(ctx->err_dev, 0, 2 * sizeof(uint32_t)));
  if (gg_status st = gg_htree_run(ctx, min_processing_time, pkt_time, proc_time, n, delay_out)) return st;
  uint32_t e = 0;
  GG_HIP(hipMemcpy(&e, ctx->err_dev, sizeof(e), hipMemcpyDeviceToHost));
  if (e & GG_DERR_RANGE) return gg_fail(GG_ERR_UNSUPPORTED, "processing time 0");
  return check_device_errors(ctx);
}

gg_status gg_shard_map(uint32_t num_tiles, uint32_t num_shards, uint32_t* tile_shard)
{
  if (!tile_shard) return gg_fail(GG_ERR_INVALID, "NULL argument");
  if (num_shards == 0 || num_shards > num_tiles) return gg_fail(GG_ERR_INVALID, "num_shards %u for %u tiles", num_shards, num_tiles);
  const int T = (int)num_tiles, K = (int)num_shards;
  const int W = (int)floor(sqrt((double)T)), H = (int)ceil(1.0 * T / W);
  if (W * H != T) {                                   // not a mesh: contiguous tile ranges
    for (int t = 0; t < T; ++t) tile_shard[t] = (uint32_t)(((uint64_t)t * K) / T);
    return GG_OK;
  }
  // NetworkModelEMeshHopByHop::computeProcessToTileMapping (hop_by_hop.cc:367-433):
  // a pw x ph grid of blocks over the first mesh_height_l rows, the remaining
  // processes side by side in the rows below
  std::vector<uint32_t> m((size_t)T, ~0u);
  const int pw = (int)floor(sqrt((double)K)), ph = (int)floor(1.0 * K / pw);
  const int hl = (int)((1.0 * H * pw * ph) / K);
  auto fill = [&](int bx, int by, int sx, int sy, uint32_t k) {
    for (int y = by; y < by + sy; ++y)
      for (int x = bx; x < bx + sx; ++x) m[(size_t)y * W + x] = k;
  };
  for (int i = 0; i < pw; ++i)
    for (int j = 0; j < ph; ++j) {
      const int bsx = W / pw, bsy = hl / ph;
      fill(i * bsx, j * bsy, i == pw - 1 ? W - (pw - 1) * bsx : bsx, j == ph - 1 ? hl - (ph - 1) * bsy : bsy,
           (uint32_t)(i + j * pw));
    }
  const int left = K - pw * ph;
  for (int i = pw * ph; i < K; ++i) {
    const int bsx = W / left;
    fill((i - pw * ph) * bsx, hl, i == K - 1 ? W - (left - 1) * bsx : bsx, H - hl, (uint32_t)i);
  }
  std::vector<char> seen((size_t)K, 0);
  for (int t = 0; t < T; ++t) {
    if (m[t] >= (uint32_t)K) return gg_fail(GG_ERR_INVALID, "no shard map for %u tiles in %u shards", num_tiles, num_shards);
    seen[m[t]] = 1;
  }
  for (int k = 0; k < K; ++k)
    if (!seen[k]) return gg_fail(GG_ERR_INVALID, "shard %d of %u is empty", k, num_shards);
  std::memcpy(tile_shard, m.data(), sizeof(uint32_t) * T);
  return GG_OK;
}

float gg_kernel_time_ms(gg_ctx* ctx, const char* kernel)
{
  if (!ctx || !kernel) return -1.0f;
  for (gg_timer& t : ctx->timers) {
    if (t.name == kernel && t.valid) {
      if (hipEventSynchronize(t.stop) != hipSuccess) return -1.0f;
      float ms = -1.0f;
      if (hipEventElapsedTime(&ms, t.start, t.stop) != hipSuccess) return -1.0f;
      return ms;
    }
  }
  return -1.0f;
}

void gg_set_timing(gg_ctx* ctx, int enabled) { if (ctx) ctx->timing = enabled < 0 ? 0 : enabled; }

gg_status gg_kernel_stats(gg_ctx* ctx, const char* kernel, double* total_ms, uint64_t* launches)
{
  if (!ctx || !kernel || !total_ms || !launches) return gg_fail(GG_ERR_INVALID, "NULL argument");
  if (gg_coh_kernel_stats(ctx, kernel, total_ms, launches) != GG_OK)
    return gg_fail(GG_ERR_INVALID, "no launch statistics for kernel '%s'", kernel);
  return GG_OK;
}

gg_status gg_gen_uniform_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin, uint32_t tiles,
                               uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift, void* stream)
{
  if (!addr_dev || !meta_dev || lines_log2 > 40) return gg_fail(GG_ERR_INVALID, "bad generator arguments");
  const uint64_t n = (uint64_t)tiles * per_tile;
  if (n == 0) return GG_OK;
  hipLaunchKernelGGL(k_gen_uniform, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     addr_dev, meta_dev, tile_begin, tiles, per_tile, first, lines_log2, base_shift);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

gg_status gg_gen_stress_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin, uint32_t tiles,
                              uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift,
                              uint32_t num_tiles, uint32_t pool_lines, uint32_t pool_frac256, void* stream)
{
  if (!addr_dev || !meta_dev || lines_log2 > 31 || pool_frac256 > 256 || (uint64_t)tile_begin + tiles > (1ull << 17) ||
      pool_lines > (1u << 24))
    return gg_fail(GG_ERR_INVALID, "gg_gen_stress_trace: bad arguments");
  const uint64_t n = (uint64_t)tiles * per_tile;
  if (!n) return GG_OK;
  hipLaunchKernelGGL(k_gen_stress, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     addr_dev, meta_dev, tile_begin, tiles, per_tile, first, lines_log2, base_shift, num_tiles,
                     pool_lines, pool_frac256);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

gg_status gg_gen_hotspot_trace(uint64_t* addr_dev, uint32_t* meta_dev, uint32_t tile_begin, uint32_t tiles,
                               uint64_t per_tile, uint64_t first, uint32_t lines_log2, uint32_t base_shift,
                               uint32_t hot_lines, uint32_t hot_frac256, void* stream)
{
  if (!addr_dev || !meta_dev || lines_log2 > 31 || hot_frac256 > 256 || (uint64_t)tile_begin + tiles > (1ull << 17))
    return gg_fail(GG_ERR_INVALID, "bad generator arguments");
  const uint64_t n = (uint64_t)tiles * per_tile;
  if (n == 0) return GG_OK;
  hipLaunchKernelGGL(k_gen_hotspot, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     addr_dev, meta_dev, tile_begin, tiles, per_tile, first, lines_log2, base_shift, hot_lines,
                     hot_frac256);
  GG_HIP(hipGetLastError());
  return GG_OK;
}

}  // extern "C"
