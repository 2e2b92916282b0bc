// gg_replay — host driver: replays a line-access trace through the MI355X
// private-cache backend and prints the per-tile "Cache Summary" blocks in the
// reference's sim.out format (Cache::outputSummary, cache.cc:419-477).
//
//   gg_replay --tiles T --per-tile N [--lines-log2 L] [--batches B] [--l2-assoc A]
//       synthetic configs[1] trace, generated on the host
//   gg_replay --tiles T --trace FILE [--batches B]
//       FILE: little-endian records {u32 tile, u32 meta, u64 byte address}
//   gg_replay --coherent --tiles T --per-tile N [--hot-lines H] [--net hop_counter|hop_by_hop|magic]
//       coherent mode (MSI directory + DRAM + NoC, gg_coherent_run) on the
//       configs[2..4] hotspot trace generated on the device; prints every
//       tile's memory block (MemoryManager::outputSummary) and memory-network
//       block (Network::outputSummary, network.cc:79-89, the Memory network)
//   gg_replay --coherent ... --shards K --ranks W --rank R --id-file FILE
//       the same over W processes (one per GPU, device R mod #devices), rank R
//       owning logical shards [R*K/W, (R+1)*K/W): RCCL communicator from the
//       unique id rank 0 writes to FILE, the run by gg_coherent_run_ranks
//       (gg_round_exchange at every quantum boundary), the statistics summed
//       over ranks and printed by rank 0
//   gg_replay --coherent ... --table
//       the tiles' summaries as TileManager::outputSummary's table
//       (tile_manager_summary.cc:135-244) instead of one block per tile
//   gg_replay --format-table FILE...
//       that table for per-tile summary texts read from the files
//   gg_replay --tiles T --net M --route FILE
//       NetworkModel::routePacket (the host mirror, broadcasts through the
//       hop-by-hop broadcast tree) on a packet file; hops + network summaries
//   gg_replay --summary-selftest
//       prints writeCacheSummary() for fixed counters (no GPU needed)
//   gg_replay --mosi-summary FILE TILES
//       prints "Tile t:" + the MOSI L2 / directory controller blocks of the
//       [TILES][GG_NUM_PROTO_STATS] counters in FILE (no GPU needed)
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "graphite_host.hpp"

using namespace graphite_amd;

static uint64_t splitmix_at(uint64_t seed, uint64_t i)
{
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv)
{
  uint32_t tiles = 4, lines_log2 = 15, batches = 1, l2_assoc = 8, hot_lines = 64, net = GG_NET_EMESH_HOP_COUNTER;
  bool coherent = false, table = false;
  uint64_t per_tile = 100000;
  std::string trace, id_file;
  int ranks = 1, rank = 0;
  uint32_t shards = 1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); } return argv[++i]; };
    if (a == "--tiles") tiles = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--per-tile") per_tile = std::strtoull(next(), nullptr, 0);
    else if (a == "--lines-log2") lines_log2 = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--batches") batches = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--l2-assoc") l2_assoc = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--trace") trace = next();
    else if (a == "--coherent") coherent = true;
    else if (a == "--table") table = true;
    else if (a == "--format-table") {
      // TileManager::outputSummary's table of the per-tile summary texts in the files that follow
      std::vector<std::string> per_tile;
      for (++i; i < argc; ++i) {
        std::ifstream f(argv[i], std::ios::binary);
        if (!f) { std::fprintf(stderr, "cannot open %s\n", argv[i]); return 2; }
        per_tile.push_back(std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>()));
      }
      std::cout << formatTileSummaries(per_tile);
      return 0;
    }
    else if (a == "--route") {
      // NetworkModel::routePacket on a packet file {u32 src, u32 dst (0xDEADBABE = broadcast),
      // u32 bits, u32 0, u64 time_ps} under --net (given before --route): one line per hop
      // "tile time zero_load contention", then each tile's Network::outputSummary
      std::ifstream f(next(), std::ios::binary);
      if (!f) { std::fprintf(stderr, "cannot open packet file\n"); return 2; }
      std::vector<char> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      std::vector<NetPacket> pk(raw.size() / 24);
      for (size_t k = 0; k < pk.size(); ++k) {
        uint32_t w[4]; uint64_t t;
        std::memcpy(w, &raw[24 * k], 16); std::memcpy(&t, &raw[24 * k + 16], 8);
        pk[k].sender = w[0]; pk[k].receiver = w[1]; pk[k].modeled_length_bits = w[2]; pk[k].time_ps = t;
      }
      gg_config cfg;
      gg_config_default(&cfg, tiles);
      cfg.net_model = net;
      Backend be(cfg);
      graphite_amd::NetworkModel nm(be);
      std::vector<Hop> hops;
      nm.routePackets(pk, hops);
      for (const Hop& h : hops)
        std::printf("%u %llu %llu %llu\n", h.next_tile_id, (unsigned long long)h.time_ps,
                    (unsigned long long)h.zero_load_delay_ps, (unsigned long long)h.contention_delay_ps);
      std::vector<uint64_t> nc((size_t)tiles * GG_NUM_NET_COUNTERS);
      check(gg_noc_get_counters(be.ctx(), nc.data()), "gg_noc_get_counters");
      for (uint32_t t = 0; t < tiles; ++t)
        writeNetworkSummary(std::cout, &nc[(size_t)t * GG_NUM_NET_COUNTERS], cfg.frequency_ghz, cfg.net_model,
                            cfg.net_model == GG_NET_EMESH_HOP_BY_HOP);
      return 0;
    }
    else if (a == "--shards") shards = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--ranks") ranks = std::atoi(next());
    else if (a == "--rank") rank = std::atoi(next());
    else if (a == "--id-file") id_file = next();
    else if (a == "--hot-lines") hot_lines = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--net") {
      const std::string n = next();
      if (n == "hop_counter") net = GG_NET_EMESH_HOP_COUNTER;
      else if (n == "hop_by_hop") net = GG_NET_EMESH_HOP_BY_HOP;
      else if (n == "magic") net = GG_NET_MAGIC;
      else { std::fprintf(stderr, "unknown network %s\n", n.c_str()); return 2; }
    }
    else if (a == "--mosi-summary" && i + 2 < argc) {
      std::ifstream f(argv[i + 1], std::ios::binary);
      const uint32_t T = (uint32_t)atoi(argv[i + 2]);
      std::vector<uint64_t> ps((size_t)T * GG_NUM_PROTO_STATS);
      f.read(reinterpret_cast<char*>(ps.data()), (std::streamsize)(ps.size() * 8));
      if (!f) { fprintf(stderr, "cannot read %s\n", argv[i + 1]); return 1; }
      for (uint32_t t = 0; t < T; ++t) {
        std::cout << "Tile " << t << ":\n";
        writeMosiL2CntlrSummary(std::cout, &ps[(size_t)t * GG_NUM_PROTO_STATS]);
        writeMosiDirectoryCntlrSummary(std::cout, &ps[(size_t)t * GG_NUM_PROTO_STATS]);
      }
      return 0;
    } else if (a == "--summary-selftest") {
      const uint64_t c1[GG_NUM_CACHE_COUNTERS] = {1000, 250, 700, 150, 300, 100, 240, 0, 2600, 900, 760, 1250};
      const uint64_t c2[GG_NUM_CACHE_COUNTERS] = {250, 180, 150, 110, 100, 70, 120, 45, 700, 600, 190, 480};
      const uint64_t z[GG_NUM_CACHE_COUNTERS] = {0};
      writeCacheSummary(std::cout, "L1-D", c1, false);
      writeCacheSummary(std::cout, "L2", c2, true);
      writeCacheSummary(std::cout, "L2", z, true);
      return 0;
    } else if (a == "--net-summary-selftest") {
      uint64_t nc[GG_NUM_NET_COUNTERS] = {0};
      nc[GG_NC_PACKETS_SENT] = 70; nc[GG_NC_FLITS_SENT] = 430; nc[GG_NC_BITS_SENT] = 24530;
      nc[GG_NC_PACKETS_RECEIVED] = 66; nc[GG_NC_FLITS_RECEIVED] = 400; nc[GG_NC_BITS_RECEIVED] = 23000;
      nc[GG_NC_TOTAL_LATENCY_PS] = 1234567; nc[GG_NC_TOTAL_CONTENTION_PS] = 45001;
      nc[GG_NC_BUFFER_WRITES] = 1720; nc[GG_NC_BUFFER_READS] = 1720; nc[GG_NC_SWITCH_ALLOC] = 280;
      nc[GG_NC_CROSSBAR] = 1720; nc[GG_NC_LINK_TRAVERSALS] = 1720;
      const uint64_t z[GG_NUM_NET_COUNTERS] = {0};
      writeNetworkSummary(std::cout, nc, 1.0, GG_NET_EMESH_HOP_COUNTER);
      writeNetworkSummary(std::cout, nc, 2.5, GG_NET_EMESH_HOP_BY_HOP);
      nc[GG_NC_ROUTER_CONTENTION_CYCLES] = 913; nc[GG_NC_ROUTER_PACKETS] = 280; nc[GG_NC_ANALYTICAL_REQUESTS] = 3;
      const uint64_t util[5] = {120, 0, 450, 77, 1000}, last[5] = {9000, 0, 12345, 8000, 40001};
      for (int p = 0; p < 5; ++p) { nc[GG_NC_PORT_UTILIZED_CYCLES + p] = util[p]; nc[GG_NC_PORT_LAST_CYCLES + p] = last[p]; }
      writeNetworkSummary(std::cout, nc, 1.0, GG_NET_EMESH_HOP_BY_HOP, true);
      writeNetworkSummary(std::cout, z, 1.0, GG_NET_MAGIC);
      return 0;
    } else if (a == "--mem-summary-selftest") {
      uint64_t st[GG_NUM_TILE_STATS] = {0};
      st[GG_CT_DIR_ACCESSES] = 5123; st[GG_CT_DIR_EVICTIONS] = 17; st[GG_CT_DIR_BACK_INVALIDATIONS] = 9;
      st[GG_CT_DRAM_ACCESSES] = 321; st[GG_CT_DRAM_LATENCY_NS] = 40417; st[GG_CT_DRAM_QUEUE_DELAY_NS] = 1537;
      st[GG_CT_DRAM_QUEUE_REQUESTS] = 321; st[GG_CT_DRAM_QUEUE_ANALYTICAL] = 7;
      st[GG_CT_DRAM_QUEUE_UTILIZED_NS] = 4173; st[GG_CT_DRAM_QUEUE_LAST_NS] = 90211;
      uint64_t cc[2 * GG_NUM_CACHE_COUNTERS] = {1000, 250, 700, 150, 300, 100, 240, 0, 2600, 900, 760, 1250,
                                                250, 180, 150, 110, 100, 70, 120, 45, 700, 600, 190, 480};
      const uint64_t z[GG_NUM_TILE_STATS] = {0};
      gg_config c;
      gg_config_default(&c, 64);
      writeMemorySummary(std::cout, c, st, cc);                       // auto sizing, history_tree
      gg_config_default(&c, 1024);
      c.dram_queue_model_type = GG_QM_HISTORY_LIST;
      writeDramSummary(std::cout, st, true, c.dram_queue_model_type);
      writeDirectorySummary(std::cout, z, directorySizing(c));
      c.dir_total_entries = 4096; c.dir_access_cycles = 3;
      writeDramSummary(std::cout, z, false, GG_QM_HISTORY_TREE);       // 0 accesses, no queue block
      writeDirectorySummary(std::cout, st, directorySizing(c));
      writeDramSummary(std::cout, st, true, GG_QM_BASIC);
      return 0;
    } else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  if (coherent) {
    ncclComm_t comm = nullptr;
    try {
      gg_config cfg;
      gg_config_default(&cfg, tiles);
      cfg.l2_assoc = l2_assoc;
      cfg.net_model = net;
      cfg.num_shards = shards;
      if (!id_file.empty()) {
        // one process per GPU: the RCCL communicator of `ranks` processes
        if (rank < 0 || rank >= ranks || shards % (uint32_t)ranks) {
          std::fprintf(stderr, "gg_replay: rank %d of %d, %u shards\n", rank, ranks, shards);
          return 2;
        }
        int ndev = 1;
        hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
        cfg.device = rank % ndev;
        hip_check(hipSetDevice(cfg.device), "hipSetDevice");
        ncclUniqueId id;
        if (rank == 0) {
          if (ncclGetUniqueId(&id) != ncclSuccess) { std::fprintf(stderr, "gg_replay: ncclGetUniqueId\n"); return 1; }
          const std::string tmp = id_file + ".tmp";
          std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char*>(&id), sizeof(id));
          std::rename(tmp.c_str(), id_file.c_str());
        } else {
          for (int w = 0;; ++w) {
            std::ifstream f(id_file, std::ios::binary);
            if (f && f.read(reinterpret_cast<char*>(&id), sizeof(id))) break;
            if (w > 6000) { std::fprintf(stderr, "gg_replay: no RCCL id in %s\n", id_file.c_str()); return 1; }
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
          }
        }
        if (ncclCommInitRank(&comm, ranks, id, rank) != ncclSuccess) {
          std::fprintf(stderr, "gg_replay: ncclCommInitRank\n");
          return 1;
        }
        cfg.shard_begin = (uint32_t)rank * (shards / ranks);
        cfg.shard_end = ((uint32_t)rank + 1) * (shards / ranks);
      }
      Backend be(cfg);
      const uint64_t n = (uint64_t)tiles * per_tile;
      DeviceBuffer<uint64_t> addr;
      DeviceBuffer<uint32_t> meta;
      addr.resize(n); meta.resize(n);
      check(gg_gen_hotspot_trace(addr.p, meta.p, 0, tiles, per_tile, 0, lines_log2, 26, hot_lines, 51, nullptr),
            "gg_gen_hotspot_trace");
      std::vector<uint64_t> offs(tiles + 1);
      for (uint32_t t = 0; t <= tiles; ++t) offs[t] = (uint64_t)t * per_tile;
      gg_trace tr{addr.p, meta.p, offs.data(), n};
      if (comm) check(gg_coherent_run_ranks(be.ctx(), comm, &tr, nullptr, nullptr), "gg_coherent_run_ranks");
      else check(gg_coherent_run(be.ctx(), &tr, nullptr, nullptr), "gg_coherent_run");
      std::vector<uint64_t> st((size_t)tiles * GG_NUM_TILE_STATS), cc((size_t)tiles * 2 * GG_NUM_CACHE_COUNTERS),
          nc((size_t)tiles * GG_NUM_NET_COUNTERS);
      check(gg_coherent_get_stats(be.ctx(), st.data(), cc.data(), nullptr), "gg_coherent_get_stats");
      check(gg_noc_get_counters(be.ctx(), nc.data()), "gg_noc_get_counters");
      if (comm) {
        // every statistic is kept by the rank owning its tile: the node's totals are the sums
        for (std::vector<uint64_t>* v : {&st, &cc, &nc}) {
          DeviceBuffer<uint64_t> d;
          d.resize(v->size());
          hip_check(hipMemcpy(d.p, v->data(), sizeof(uint64_t) * v->size(), hipMemcpyHostToDevice), "hipMemcpy");
          if (ncclAllReduce(d.p, d.p, v->size(), ncclUint64, ncclSum, comm, nullptr) != ncclSuccess)
            throw Error(GG_ERR_STATE, "ncclAllReduce");
          hip_check(hipMemcpy(v->data(), d.p, sizeof(uint64_t) * v->size(), hipMemcpyDeviceToHost), "hipMemcpy");
        }
      }
      std::vector<std::string> per_tile;
      for (uint32_t t = 0; rank == 0 && t < tiles; ++t) {
        std::ostringstream os;
        writeTileSummary(os, cfg, &st[(size_t)t * GG_NUM_TILE_STATS], &cc[(size_t)t * 2 * GG_NUM_CACHE_COUNTERS],
                         &nc[(size_t)t * GG_NUM_NET_COUNTERS]);
        if (table) per_tile.push_back(os.str());
        else std::cout << "Tile " << t << " Summary:" << std::endl << os.str();
      }
      if (table && rank == 0) std::cout << formatTileSummaries(per_tile);
    } catch (const Error& e) {
      std::fprintf(stderr, "gg_replay: %s\n", e.what());
      if (comm) ncclCommDestroy(comm);
      return 1;
    }
    if (comm) ncclCommDestroy(comm);
    return 0;
  }
  try {
    gg_config cfg;
    gg_config_default(&cfg, tiles);
    cfg.l2_assoc = l2_assoc;
    Backend be(cfg);
    TraceReplayer rep(be);
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> recs(tiles);
    if (!trace.empty()) {
      std::ifstream f(trace, std::ios::binary);
      if (!f) { std::fprintf(stderr, "cannot open %s\n", trace.c_str()); return 2; }
      uint32_t hdr[2]; uint64_t addr;
      while (f.read((char*)hdr, 8) && f.read((char*)&addr, 8)) {
        if (hdr[0] >= tiles) { std::fprintf(stderr, "record for tile %u >= %u tiles\n", hdr[0], tiles); return 2; }
        recs[hdr[0]].push_back({addr, hdr[1]});
      }
    } else {
      for (uint32_t t = 0; t < tiles; ++t) {
        const uint64_t seed = 0x9E3779B97F4A7C15ull ^ t;
        for (uint64_t i = 0; i < per_tile; ++i) {
          const uint64_t z = splitmix_at(seed, i);
          recs[t].push_back({((uint64_t)t << 26) + ((z & ((1ull << lines_log2) - 1)) << 6),
                             ((z >> 32) % 3 == 0) ? GG_META_WRITE : 0u});
        }
      }
    }
    uint64_t misses = 0;
    for (uint32_t b = 0; b < batches; ++b) {
      for (uint32_t t = 0; t < tiles; ++t) {
        const size_t n = recs[t].size(), lo = n * b / batches, hi = n * (b + 1) / batches;
        for (size_t i = lo; i < hi; ++i)
          rep.accessSingleLine(t, (recs[t][i].second & GG_META_WRITE) != 0, recs[t][i].first);
      }
      for (uint32_t r : rep.flush()) misses += (r & GG_RES_L1_MISS) != 0;
    }
    rep.outputSummary(std::cout);
    std::cout << "L1-D misses reported per access: " << misses << std::endl;
  } catch (const Error& e) {
    std::fprintf(stderr, "gg_replay: %s\n", e.what());
    return 1;
  }
  return 0;
}
