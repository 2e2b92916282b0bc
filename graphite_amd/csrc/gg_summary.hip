// gg_summary.hip — gg_dump_summary: the sim.out text of a context's
// statistics through the C ABI (host code; the formatting is the host
// mirror's, graphite_amd/host/graphite_host.hpp, which restates
// Cache::outputSummary cache.cc:419-477, NetworkModel::outputSummary
// network_model.cc:274-316, the hop-by-hop event / contention summaries
// network_model_emesh_hop_by_hop.cc:436-486, DramPerfModel::outputSummary
// dram_perf_model.cc:131-164, DirectoryCache::outputSummary
// directory_cache.cc:350-398 and TileManager::outputSummary's table
// tile_manager_summary.cc:60-244).
#include "gg_internal.h"

#include <cstring>
#include <sstream>

#include "../host/graphite_host.hpp"

gg_status gg_dump_summary(gg_ctx* ctx, int format, char* buf, uint64_t cap, uint64_t* needed)
{
  if (!ctx || !needed) return gg_fail(GG_ERR_INVALID, "NULL argument");
  if (format != GG_SUMMARY_BLOCKS && format != GG_SUMMARY_TABLE) return gg_fail(GG_ERR_INVALID, "format %d", format);
  const gg_config& cfg = ctx->cfg;
  const uint32_t T = cfg.num_tiles;
  std::vector<uint64_t> st, cc((size_t)T * 2 * GG_NUM_CACHE_COUNTERS), nc((size_t)T * GG_NUM_NET_COUNTERS);
  const bool coherent = ctx->coh != nullptr;
  if (coherent) {
    st.resize((size_t)T * GG_NUM_TILE_STATS);
    if (gg_status e = gg_coherent_get_stats(ctx, st.data(), cc.data(), nullptr)) return e;
  } else if (gg_status e = gg_cache_get_counters(ctx, cc.data())) return e;
  if (gg_status e = gg_noc_get_counters(ctx, nc.data())) return e;
  std::vector<uint64_t> mt;
  const bool mosi = cfg.protocol == GG_PROTO_MOSI;
  std::vector<uint64_t> ps;
  if (coherent && mosi) {
    ps.resize((size_t)T * GG_NUM_PROTO_STATS);
    if (gg_status e = gg_coherent_get_protocol_stats(ctx, ps.data())) return e;
  }
  if (coherent && (((mosi || cfg.protocol >= GG_PROTO_SHL2_MSI) ? cfg.l1d_track_miss_types : cfg.l1i_track_miss_types) ||
                   cfg.l2_track_miss_types)) {
    mt.resize((size_t)T * 2 * GG_NUM_MISS_TYPES);
    if (gg_status e = gg_coherent_get_miss_types(ctx, mt.data())) return e;
  }
  std::vector<uint64_t> core;
  if (ctx->core_valid) {                       // gg_core_model_run's statistics: the "Core Summary" blocks
    core.resize((size_t)T * GG_NUM_CORE_STATS);
    if (gg_status e = gg_core_get_stats(ctx, core.data())) return e;
  }
  std::vector<uint64_t> io;
  if (ctx->io_valid) {                         // gg_iocoom_run's statistics: the iocoom "Core Summary" blocks
    io.resize((size_t)T * GG_NUM_IOCOOM_STATS);
    if (gg_status e = gg_iocoom_get_stats(ctx, io.data())) return e;
  }
  std::string text;
  try {
    std::vector<std::string> per_tile;
    std::ostringstream all;
    for (uint32_t t = 0; t < T; ++t) {
      std::ostringstream os;
      graphite_amd::writeTileSummary(os, cfg, coherent ? &st[(size_t)t * GG_NUM_TILE_STATS] : nullptr,
                                     &cc[(size_t)t * 2 * GG_NUM_CACHE_COUNTERS], &nc[(size_t)t * GG_NUM_NET_COUNTERS],
                                     core.empty() ? nullptr : &core[(size_t)t * GG_NUM_CORE_STATS],
                                     mt.empty() ? nullptr : &mt[(size_t)t * 2 * GG_NUM_MISS_TYPES],
                                     ps.empty() ? nullptr : &ps[(size_t)t * GG_NUM_PROTO_STATS],
                                     io.empty() ? nullptr : &io[(size_t)t * GG_NUM_IOCOOM_STATS]);
      if (format == GG_SUMMARY_TABLE) per_tile.push_back(os.str());
      else all << "Tile " << t << " Summary:" << std::endl << os.str();
    }
    text = format == GG_SUMMARY_TABLE ? graphite_amd::formatTileSummaries(per_tile) : all.str();
  } catch (const std::exception& e) {
    return gg_fail(GG_ERR_STATE, "summary: %s", e.what());
  }
  *needed = (uint64_t)text.size() + 1;
  if (!buf || cap < *needed) return buf ? gg_fail(GG_ERR_RANGE, "summary needs %llu bytes", (unsigned long long)*needed)
                                        : GG_OK;
  std::memcpy(buf, text.c_str(), text.size() + 1);
  return GG_OK;
}
