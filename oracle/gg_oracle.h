/*
 * gg_oracle.h — CPU restatement of the reference algorithms on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in graphite_amd/ links, loads or calls
 * this code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, as the checker / the CPU baseline.  Every function names the
 * reference file:line it restates (paths relative to nmtrmail/Graphite).
 *
 * Pinning: the history-tree queue model is pinned by the
 * reference KAT (tests/unit/history_tree/history_tree.cc:9-20); the cache
 * set / LRU / round-robin / line-info layer and the interval tree are pinned
 * by fixtures produced by the reference's own code compiled from
 * /root/reference (oracle/ref/, outputs in tests/golden/); the controller glue
 * (L1/L2 MSI private path, NoC models) is a restatement checked by those
 * fixtures where they reach and otherwise "parity unpinned" (cache.cc,
 * l1/l2_cache_cntlr.cc and the network models need Boost/Pin headers absent
 * from this image).
 */
#ifndef GG_ORACLE_H
#define GG_ORACLE_H
#include <stdint.h>
#include "../include/graphite_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- synthetic trace generators -------- */
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t i);
/* configs[1]: uniform private region of 2^lines_log2 lines per tile at
 * byte base tile << base_shift, WRITE iff ((z >> 32) % 3) == 0.             */
void oracle_gen_uniform(uint32_t tile, uint64_t first, uint64_t n,
                        uint32_t lines_log2, uint32_t base_shift,
                        uint64_t* addr, uint32_t* meta);

/* configs[2..4]: hotspot / shared-line trace with core-cycle gaps (meta bits 1..30). */
void oracle_gen_hotspot(uint32_t tile, uint64_t first, uint64_t n, uint32_t lines_log2,
                        uint32_t base_shift, uint32_t hot_lines, uint32_t hot_frac256,
                        uint64_t* addr, uint32_t* meta);

void oracle_gen_stress(uint32_t tile, uint64_t first, uint64_t n, uint32_t lines_log2, uint32_t base_shift,
                       uint32_t num_tiles, uint32_t pool_lines, uint32_t pool_frac256, uint64_t* addr, uint32_t* meta);

/* ---------------- private cache replay (mode P) ---------------------------- */
typedef struct oracle_cache oracle_cache;
oracle_cache* oracle_cache_create(const gg_config* cfg);
void          oracle_cache_destroy(oracle_cache* oc);
/* Replays tiles [tile_begin, tile_end) of a tile-major trace; result/evicted
 * may be NULL.  Returns 0 or GG_ERR_STATE where the reference would abort.  */
int  oracle_cache_run(oracle_cache* oc, const uint64_t* addr, const uint32_t* meta,
                      const uint64_t* tile_offsets, uint32_t tile_begin, uint32_t tile_end,
                      uint32_t* result, uint64_t* evicted);
void oracle_cache_counters(const oracle_cache* oc, uint64_t* out); /* [tile][2][12] */
/* The Cache quartet (cache.cc:84-241) on one tile/level. */
int  oracle_cache_get_line_info(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, gg_line_info* out);
int  oracle_cache_set_line_info(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, const gg_line_info* in);
int  oracle_cache_access_line(oracle_cache* oc, uint32_t tile, int level, uint64_t addr, int is_store);
int  oracle_cache_insert_line(oracle_cache* oc, uint32_t tile, int level, uint64_t addr,
                              const gg_line_info* in, int* eviction, uint64_t* evicted_addr,
                              gg_line_info* evicted_info);

/* ---------------- queue models ------------------------------------------- */
typedef struct oracle_htree oracle_htree;
oracle_htree* oracle_htree_create(uint64_t min_processing_time, int max_list_size, int analytical_enabled);
/* any QueueModel::create type (GG_QM_*); aux = history_list_no_interleaving
 * for history_list, basic_moving_avg for basic (gg_config fields)          */
oracle_htree* oracle_qmodel_create(uint32_t type, uint32_t aux, uint64_t min_processing_time,
                                   int max_list_size, int analytical_enabled);
void          oracle_htree_destroy(oracle_htree* h);
uint64_t      oracle_htree_delay(oracle_htree* h, uint64_t pkt_time, uint64_t processing_time);
uint64_t      oracle_htree_analytical_requests(const oracle_htree* h);
uint32_t      oracle_htree_size(const oracle_htree* h);

/* ---------------- NoC ------------------------------------------------------ */
typedef struct oracle_noc oracle_noc;
oracle_noc* oracle_noc_create(const gg_config* cfg);
void        oracle_noc_destroy(oracle_noc* on);
int  oracle_noc_route(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst,
                      const uint32_t* length_bits, const uint64_t* time_ps,
                      uint64_t* arrival_ps, uint64_t* zero_load_ps, uint64_t* contention_ps);
/* broadcast tree (dst == GG_BROADCAST): b_* = [broadcast ordinal][tile] */
int  oracle_noc_route_tree(oracle_noc* on, uint64_t n, const uint32_t* src, const uint32_t* dst,
                           const uint32_t* len, const uint64_t* time_ps,
                           uint64_t* arrival, uint64_t* zero_load, uint64_t* contention,
                           uint64_t* b_arrival, uint64_t* b_zero_load, uint64_t* b_contention);
void oracle_noc_counters(const oracle_noc* on, uint64_t* out); /* [tile][GG_NUM_NET_COUNTERS] */

/* ---------------- coherent mode (Mode C) ----------------
 * pr_l1_pr_l2_dram_directory_msi with directory, DRAM, NoC and lax-barrier
 * quanta in the canonical schedule (oracle/gg_coherent.inc).  The context
 * owns shards [cfg.shard_begin, cfg.shard_end) of cfg.num_shards.          */
typedef struct oracle_coh oracle_coh;
/* tile -> logical shard (emesh_hop_by_hop process mapping, hop_by_hop.cc:367-433) */
int  oracle_shard_map(uint32_t num_tiles, uint32_t num_shards, uint32_t* tile_shard);
oracle_coh* oracle_coh_create(const gg_config* cfg);
void        oracle_coh_destroy(oracle_coh* C);
int  oracle_coh_begin(oracle_coh* C, const uint64_t* addr, const uint32_t* meta,
                      const uint64_t* tile_offsets, uint64_t* access_out);
/* status: steps, held boundary messages, min next-access start, active tiles, blocked tiles */
int  oracle_coh_quantum(oracle_coh* C, uint64_t q, uint64_t* status);
uint64_t oracle_coh_export(oracle_coh* C, gg_cmsg* out, uint64_t cap);
int  oracle_coh_import(oracle_coh* C, const gg_cmsg* in, uint64_t n);
int  oracle_coh_run(oracle_coh* C, const uint64_t* addr, const uint32_t* meta,
                    const uint64_t* tile_offsets, uint64_t* access_out);
void oracle_coh_tile_stats(const oracle_coh* C, uint64_t* out);      /* [tile][GG_NUM_TILE_STATS] */
void oracle_coh_cache_counters(const oracle_coh* C, uint64_t* out);  /* [tile][2][12] */
void oracle_coh_net_counters(const oracle_coh* C, uint64_t* out);    /* [tile][GG_NUM_NET_COUNTERS] */
void oracle_coh_run_info(const oracle_coh* C, uint64_t* out);        /* [GG_NUM_RUN_INFO] */
void oracle_coh_miss_types(const oracle_coh* C, uint64_t* out);      /* [tile][2][GG_NUM_MISS_TYPES] */
void oracle_coh_proto_stats(const oracle_coh* C, uint64_t* out);     /* [tile][GG_NUM_PROTO_STATS] (MOSI) */
void oracle_cache_miss_types(const oracle_cache* oc, uint64_t* out); /* [tile][2][GG_NUM_MISS_TYPES] */
/* the whole run with one context per logical shard, `threads` OpenMP threads */
/* tile-parallel steps on `threads` OpenMP threads (bit-identical results) */
int  oracle_coh_set_threads(oracle_coh* C, int threads);
int  oracle_coh_run_parallel(const gg_config* cfg, int threads, const uint64_t* addr, const uint32_t* meta,
                             const uint64_t* tile_offsets, uint64_t* access_out, uint64_t* tile_stats,
                             uint64_t* cache, uint64_t* net, uint64_t* run_info);

/* Network::netSend line split of Core::initiateMemoryAccess (core.cc:167-201):
 * returns the number of line accesses [addr, addr+size) produces and writes
 * their line-aligned addresses to lines (capacity cap).                    */
uint32_t oracle_split_lines(uint64_t addr, uint32_t size, uint32_t line_size,
                            uint64_t* lines, uint32_t cap);
/* Multi-line accesses as line records (GG_META_CONT) and their per-access
 * latency / miss count (core.cc:139-266); see gg_oracle.c.                 */
uint64_t oracle_split_accesses(const uint64_t* addr, const uint32_t* size, const uint32_t* meta,
                               const uint64_t* tile_offsets, uint32_t tiles, uint32_t line,
                               uint64_t* first, uint64_t* line_addr, uint32_t* line_meta);
void oracle_combine_accesses(const uint64_t* line_out, const uint64_t* first, uint64_t n,
                             uint64_t* latency_ps, uint32_t* misses);
/* The simple core model over a coherent run's per-record access words
 * (SimpleCoreModel::handleInstruction, simple_core_model.cc:43-96); see
 * gg_oracle.c.  stats: [tiles][GG_NUM_CORE_STATS].                          */
void oracle_core_model(const uint32_t* meta, const uint64_t* access_out, const uint64_t* tile_offsets,
                       uint32_t tiles, double frequency_ghz, uint64_t* stats);
/* The iocoom core model over instruction and access streams (IOCOOMCoreModel::
 * handleInstruction, iocoom_core_model.cc:66-322; the streams of
 * gg_iocoom_run); stats: [tiles][GG_NUM_IOCOOM_STATS].  Returns -1 when the
 * streams disagree (stats of the tiles before and including the bad one).   */
int oracle_iocoom(const gg_iocoom_params* p, const gg_ins* ins, const uint64_t* ins_offsets, const uint64_t* addr,
                  const uint32_t* meta, const uint64_t* lat, const uint64_t* acc_offsets, uint32_t tiles,
                  double frequency_ghz, uint64_t* stats);

#ifdef __cplusplus
}
#endif
#endif
