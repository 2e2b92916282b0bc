// gg_internal.h — shared definitions of the MI355X backend (host + device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/graphite_gpu.h"

#define GG_WAVE 64
#define GG_NUM_XCD 8          // MI355X: 8 XCDs, workgroups dealt round-robin by blockIdx

// Packed meta byte of one cache line in the device-resident state:
//   bits 0-1 state (0 I, 1 S, 2 M), bit 2 cached_loc == L1-D (L2 only),
//   bits 3-7 replacement age (LRUReplacementPolicy::_lru_bits_vec entry).
#define GG_MS_I 0u
#define GG_MS_S 1u
#define GG_MS_M 2u
#define GG_M_STATE(b) ((b) & 3u)
#define GG_M_LOC(b) (((b) >> 2) & 1u)
#define GG_M_AGE(b) ((b) >> 3)
#define GG_M_MAKE(st, loc, age) ((uint32_t)(st) | ((uint32_t)(loc) << 2) | ((uint32_t)(age) << 3))

#define GG_L1_INV_TAG (~0ull)     // CacheLineInfo invalid tag (cache_line_info.h:21-22)
#define GG_L2_INV_TAG 0xFFFFFFFFu // compressed L2 tag (line >> log2(L2 sets)); 2^32-1 is out of range

// Error bits of the device-side error word (ctx->err_dev).
#define GG_DERR_RANGE 1u   // address beyond the compressed-tag range
#define GG_DERR_STATE 2u   // the reference would LOG_ASSERT_ERROR on this state
#define GG_DERR_CAP 4u     // a device-side capacity (messages, queues, inbox) was exceeded
#define GG_DERR_BARRIER 8u // a BARRIER record (GG_META_BARRIER) reached a path that has no barriers (Mode P)

// Geometry derived from gg_config (cache.cc:44, cache_hash_fn.h:11).
struct gg_geom {
  uint32_t tiles;
  uint32_t log_line;
  uint32_t u1;        // L1-D sets = units per tile
  uint32_t log_u1;
  uint32_t a1;        // L1-D ways
  uint32_t l2_sets;
  uint32_t log_l2;
  uint32_t s2;        // L2 sets per unit (l2_sets / u1)
  uint32_t a2;        // L2 ways
  uint32_t mw;        // u64 meta words per L2 set ((a2 + 7) / 8)
  uint32_t pol1, pol2;
  uint64_t units;     // tiles * u1
  uint64_t addr_limit;  // first byte address whose L2 tag no longer fits 32 bits
};

// Device-resident cache state, structure of arrays indexed [field][unit] so a
// wave of 64 consecutive units loads/stores it coalesced.
struct gg_cache_state {
  uint64_t* l1_tag;   // [a1][units]      line address or ~0
  uint64_t* l1_meta;  // [units]          byte w = meta of way w
  uint8_t*  l1_rr;    // [units]          RoundRobin index
  uint32_t* l2_tag;   // [s2*a2][units]   line >> log2(l2_sets) or 2^32-1
  uint64_t* l2_meta;  // [s2*mw][units]   byte (w%8) of word w/8
  uint8_t*  l2_rr;    // [s2][units]
  uint64_t* counters; // [tiles][2][GG_NUM_CACHE_COUNTERS]
};

struct gg_timer {
  std::string name;
  hipEvent_t start = nullptr, stop = nullptr;
  bool valid = false;
};

struct gg_noc_state;
struct gg_coh_state;

struct gg_ctx {
  gg_config cfg;
  gg_geom g;
  int device = 0;
  int num_cus = 256;
  hipStream_t last_stream = nullptr;
  gg_cache_state cs{};
  uint32_t* err_dev = nullptr;
  // batch scratch (grown on demand)
  uint64_t* sh_key = nullptr;    // sharded records (slot order): line address | write bit
  uint32_t* sh_res = nullptr;    // replay results in slot order
  uint64_t* sh_ev = nullptr;     // evicted L2 line addresses in slot order (only when requested)
  uint64_t  sh_cap = 0, sh_res_cap = 0, sh_ev_cap = 0;
  uint32_t* rec_slot = nullptr;  // [records] slot of each program-order record (written by the scatter)
  uint64_t  rec_cap = 0;
  uint32_t* chunk_cnt = nullptr; // [chunks][u1]
  uint32_t* chunk_tile = nullptr;
  uint64_t* chunk_start = nullptr;
  uint32_t* chunk_len = nullptr;
  uint64_t  chunk_cap = 0;
  uint32_t* unit_len = nullptr;  // [units]
  uint64_t* unit_base = nullptr; // [units] slot of the unit's record 0 (records contiguous, padded to 8)
  uint64_t* total_dev = nullptr; // slots of the sharded layout
  uint64_t* tile_off_dev = nullptr; // [tiles+1]
  std::vector<uint32_t> h_chunk_tile, h_chunk_len;
  std::vector<uint64_t> h_chunk_start;
  // NoC
  gg_noc_state* noc = nullptr;
  // coherent mode (gg_coherent.hip), allocated on first use
  gg_coh_state* coh = nullptr;
  // replay kernel choice: 0 = lean when instantiated (default), 1 = generic
  int replay_variant = 0;
  // timing
  int timing = 0;                // gg_set_timing: 0 off, 1 sampled coherent launches, 2 every launch
  std::vector<gg_timer> timers;
  // core timing (gg_core.hip): [tiles][GG_NUM_CORE_STATS] and its task list
  uint64_t* core_dev = nullptr;
  void* core_tasks = nullptr;
  uint64_t core_task_cap = 0;
  bool core_valid = false;
  // the iocoom core model (gg_core.hip): [tiles][GG_NUM_IOCOOM_STATS], the
  // two offset lists [2][tiles + 1] and the stream-check word
  uint64_t* io_stats = nullptr;
  uint64_t* io_offs = nullptr;
  uint32_t* io_err = nullptr;
  bool io_valid = false;
  // multi-rank round buffers (gg_round.hip), freed by gg_destroy
  void* round = nullptr;
  void (*round_free)(void*) = nullptr;
};
inline void* gg_round_state(gg_ctx* ctx) { return ctx->round; }
inline void gg_round_state_set(gg_ctx* ctx, void* p, void (*f)(void*)) { ctx->round = p; ctx->round_free = f; }

// error reporting (gg_capi.hip)
gg_status gg_fail(gg_status code, const char* fmt, ...);
gg_status gg_hip_check(hipError_t e, const char* what);
#define GG_HIP(x) do { hipError_t _e = (x); if (_e != hipSuccess) return gg_hip_check(_e, #x); } while (0)

// timing helpers (gg_capi.hip)
void gg_timer_begin(gg_ctx* ctx, const char* name, hipStream_t s);
void gg_timer_end(gg_ctx* ctx, const char* name, hipStream_t s);

// cache path (gg_cache.hip)
gg_status gg_cache_state_alloc(gg_ctx* ctx);
void      gg_cache_state_free(gg_ctx* ctx);
gg_status gg_cache_state_reset(gg_ctx* ctx, hipStream_t s);
gg_status gg_cache_run_batch(gg_ctx* ctx, const gg_trace* tr, uint32_t* result, uint64_t* evicted, hipStream_t s);
gg_status gg_cache_quartet(gg_ctx* ctx, int op, uint32_t tile, int level, uint64_t addr,
                           const gg_line_info* in, gg_line_info* out, int* eviction, uint64_t* ev_addr);

// NoC path (gg_noc.hip)
gg_status gg_noc_alloc(gg_ctx* ctx);
void      gg_noc_free(gg_ctx* ctx);
gg_status gg_noc_reset(gg_ctx* ctx, hipStream_t s);
gg_status gg_noc_run(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out, hipStream_t s);
gg_status gg_noc_tree(gg_ctx* ctx, const gg_packets* pk, const gg_packet_out* out, const gg_packet_out* bout,
                      uint64_t nb, hipStream_t s);
gg_status gg_noc_counters(gg_ctx* ctx, uint64_t* out);
// core timing (gg_core.hip)
void      gg_core_free(gg_ctx* ctx);
// coherent path (gg_coherent.hip)
void      gg_coh_free(gg_ctx* ctx);
gg_status gg_htree_run(gg_ctx* ctx, uint64_t min_proc, const uint64_t* t, const uint64_t* p, uint64_t n, uint64_t* d);
gg_status gg_coh_kernel_stats(gg_ctx* ctx, const char* name, double* total_ms, uint64_t* launches);
uint64_t  gg_coherent_msg_cap(gg_ctx* ctx);     // records a quantum boundary can hold (after gg_coherent_begin)
// the quantum steps and the per-rank slot exchange of gg_round_exchange (gg_coherent.hip)
gg_status gg_coh_steps_async(gg_ctx* ctx, uint64_t q, uint32_t k0, uint32_t n);
gg_status gg_coh_round_tail(gg_ctx* ctx, gg_cmsg* slots, uint32_t world, uint32_t per_rank, uint64_t region,
                            uint32_t host_err, uint64_t* dv_own);
gg_status gg_coh_round_import(gg_ctx* ctx, uint64_t q, const gg_cmsg* send, const gg_cmsg* recv, uint32_t world,
                              uint32_t self, uint64_t region, uint64_t slot, const uint64_t* dv_all, uint64_t* counts);
void      gg_coh_harvest(gg_ctx* ctx);
constexpr int kRoundWords = 8;          // a rank's round status words (RW_* in gg_coherent.hip)
gg_status gg_coh_import_slots(gg_ctx* ctx, const gg_cmsg* slots, uint32_t world, uint64_t region, uint64_t lo,
                              uint64_t hi, bool first, const uint64_t* skip_if_dev);
gg_status gg_coh_check(gg_ctx* ctx);
uint64_t  gg_coh_generation(gg_ctx* ctx);    // bumped by every gg_coherent_begin (0: none yet)
