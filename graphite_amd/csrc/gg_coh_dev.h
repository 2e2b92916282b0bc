// gg_coh_dev.h — the coherent ("Mode C") path's device side, shared by the
// step (gg_coh_step.hip), walker (gg_coh_walk.hip) and host (gg_coherent.hip)
// translation units.  The kernels themselves live in those units; the host
// launches them through the launchers declared at the end.
#pragma once
// gg_coherent.hip — the coherent ("Mode C") path on MI355X (gfx950):
// pr_l1_pr_l2_dram_directory_msi with the DRAM directory, DRAM controller,
// ShmemPerfModel clock, memory network and lax-barrier quanta, in the
// canonical step schedule of DESIGN.md §4.
//
// Reference (nmtrmail/Graphite, common/tile/memory_subsystem/):
//   pr_l1_pr_l2_dram_directory_msi/l1_cache_cntlr.cc:89-305   L1 state machine
//   pr_l1_pr_l2_dram_directory_msi/l2_cache_cntlr.cc:74-527   L2 state machine
//   pr_l1_pr_l2_dram_directory_msi/dram_directory_cntlr.cc:43-550  MSI directory
//   cache/directory_cache.cc:102-348                          DirectoryCache
//   directory_schemes/directory_entry_full_map.cc:18-86       full-map sharers
//   dram_cntlr.cc:37-74, performance_models/dram_perf_model.cc:75-116  DRAM
//   performance_models/shmem_perf_model.cc:16-45              per-tile clock
//   common/network/models/network_model_emesh_hop_by_hop.cc:146-264  hop-by-hop
//   common/network/components/router/router_model.cc:52-108    output ports
//
// Execution model.  ONE WAVE PER TILE.  A tile's controllers are sequential
// by construction (the per-tile lock of memory_manager.cc:78-120), so the
// whole wave runs the tile's control flow in lockstep with identical values
// on every lane; the lanes split the work wherever the data is wide:
//   * a cache set: lane w holds way w (tag + meta byte); the hit is a ballot,
//     the LRU victim a ballot + ffs, the age update lane-parallel;
//   * a directory set: lane i checks way i; the replacement candidate is a
//     wave min over (sharers, way) of the ways with no queued request;
//   * a full-map sharer vector: lane k holds word k; an INV_REQ fan-out is a
//     popcount prefix scan and every lane writes its word's messages;
//   * the request FIFO (LDS) and the DRAM / router queues (LDS images of the
//     flat interval list of gg_dev.h): lane-parallel scans and shifts;
//   * the inbox: keys in LDS, channel prefix-max and ranks lane-parallel.
// Plain stores in the uniform parts are made by every lane (same address,
// same value), so each lane reads back its own writes; lane-parallel stores
// touch only data the same lane reads again, or are followed by a
// workgroup barrier (one wave = one workgroup) before other lanes read them.
//
// Step: k_c_step, one launch, wave per owned tile:
//   (hop-by-hop) the SELF output port + receive of the packets that reached
//   the tile in the previous step, in (time, key) order;
//   the inbox in the reference's per-channel FIFO order, channels merged by
//   (arrival, sender);  the trace up to the lax barrier or the next miss;
//   publish: hop counter / magic route every record (closed form) into its
//   receiver's inbox list or the quantum-boundary buffer; hop-by-hop sends
//   the tile's packets through its injection port in (time, key) order and
//   onto the list of the X (or Y) chain segment they enter.
// Hop-by-hop adds k_c_walk for the X segments, then for the Y segments: one
// wave per run of one row (column) inside one logical shard walks that
// run's packets in (time, key) order through the output-port queues (LDS
// images), hands packets that finish the run to the next segment list or to
// their destination's SELF list, and holds packets whose next router lies in
// another logical shard for the quantum boundary (gg_cmsg.hop).
#include "gg_dev.h"

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <vector>

#ifndef GG_COH_DIAG
#define GG_COH_DIAG 0
#endif
// a diagnostics pointer of CS: the pointer in a diagnostics build, a null
// constant otherwise (the hooks compile out wherever S lives)
#define DG(x) (GG_COH_DIAG ? (x) : nullptr)

namespace ggc {
using namespace gg;

enum { M_EX_REQ = GG_MSG_EX_REQ, M_SH_REQ = GG_MSG_SH_REQ, M_INV_REQ = GG_MSG_INV_REQ,
       M_FLUSH_REQ = GG_MSG_FLUSH_REQ, M_WB_REQ = GG_MSG_WB_REQ, M_EX_REP = GG_MSG_EX_REP,
       M_SH_REP = GG_MSG_SH_REP, M_INV_REP = GG_MSG_INV_REP, M_FLUSH_REP = GG_MSG_FLUSH_REP,
       M_WB_REP = GG_MSG_WB_REP, M_NULLIFY_REQ = GG_MSG_NULLIFY_REQ };
enum { DS_UNCACHED = 0, DS_SHARED = 1, DS_MODIFIED = 2, DS_OWNED = 3 /* MOSI */ };
enum { ST_I = 0, ST_S = 1, ST_M = 2, ST_O = 3 /* MOSI */ };   // meta byte bits 0-1
enum { M_UPGRADE_REP = GG_MSG_UPGRADE_REP, M_IFC_REQ = GG_MSG_INV_FLUSH_COMBINED_REQ };
enum { M_DRAM_FETCH_REQ = GG_MSG_DRAM_FETCH_REQ, M_DRAM_STORE_REQ = GG_MSG_DRAM_STORE_REQ,   // pr_l1_sh_l2_msi
       M_DRAM_FETCH_REP = GG_MSG_DRAM_FETCH_REP,
       M_DOWNGRADE_REQ = GG_MSG_DOWNGRADE_REQ, M_SH_REP_EX = GG_MSG_SH_REP_EX,                  // pr_l1_sh_l2_mesi
       M_DOWNGRADE_REP = GG_MSG_DOWNGRADE_REP };
constexpr uint32_t ST_E = ST_O;           // MESI's EXCLUSIVE L1 lines take the MOSI OWNED code (protocols never mix)
enum { P_SELF = 0, P_LEFT, P_RIGHT, P_DOWN, P_UP, P_INJ };   // network_model_emesh_hop_by_hop.h:41-48 (+ injection)
#define INV_ADDR (~0ull)
#define NO_ENT (-0x7fffffff)

__device__ __forceinline__ bool to_directory(uint32_t t)
{
  return t == M_EX_REQ || t == M_SH_REQ || t == M_INV_REP || t == M_FLUSH_REP || t == M_WB_REP;
}
__device__ __forceinline__ bool has_data(uint32_t t)
{
  return t == M_EX_REP || t == M_SH_REP || t == M_FLUSH_REP || t == M_WB_REP ||
         t == M_DRAM_STORE_REQ || t == M_DRAM_FETCH_REP ||          // …sh_l2_msi/shmem_msg.cc:128-140
         t == M_SH_REP_EX;                                          // (MESI's DOWNGRADE_REP carries no data buffer)
}
// modeled length class of a message (ShmemMsg::getModeledLength, shmem_msg.cc:100-125,
// …mosi/shmem_msg.cc:122-151): 0 request, 1 with a cache line, 2 MOSI
// INV_FLUSH_COMBINED_REQ (+ the single receiver's tile id)
__device__ __forceinline__ uint32_t len_class(uint32_t t) { return has_data(t) ? 1u : t == M_IFC_REQ ? 2u : 0u; }

struct DEnt { uint64_t addr; int32_t owner; uint16_t dstate; uint16_t nsh; };   // 16 B
struct HMsg { uint64_t addr, arrival_ps; uint32_t type, src, requester, single_rx; };   // the fields a handler reads
// a tile's step state (trace position, clock, pending access, blocking,
// sequence, replaced entries, request FIFO length): one line, one pointer
struct TileSt { uint64_t rec, rec_end, clk, pend_start, out_addr, out_time; uint32_t blocked, seq, nrep, nrq; };
static_assert(sizeof(TileSt) == 64, "one 64-B line per tile");
struct CReq { uint64_t addr, time; uint32_t type, requester; };                 // 24 B
// MOSI: the rest of a ShmemReq (…mosi/shmem_req.h:14-66) beside its FIFO slot
// (CReq::time is its _processing_finish_time there)
struct CReqX { uint64_t arrival, start; uint32_t ds0, upg; int32_t sharer; uint32_t pad; };   // 32 B
constexpr uint32_t kCdl = 64;          // MOSI: the directory's cached data list, entries per tile
// MOSI: a directory entry's Random (drand48_r state X) is stored XOR its seed
// state, so zeroed memory is a freshly created entry (misc/random.h:14-23)
constexpr uint64_t kRng0 = ((uint64_t)(uint32_t)GG_MOSI_RNG_SEED << 16) | 0x330Eu;
// address-space-typed pointers (a generic pointer whose origin the compiler
// cannot see compiles to flat accesses)
#define GG_LDS __attribute__((address_space(3)))
#define GG_GLB __attribute__((address_space(1)))
// CS's pointers are global in the device pass (GG_DP), so every access derived
// from them compiles to global_* instead of flat_* (a flat access counts in
// both vmcnt and lgkmcnt: each wait for a scalar or LDS result would also wait
// for it).  The host pass sees plain pointers; the layout is the same.
#if defined(__HIP_DEVICE_COMPILE__)
#define GG_DP __attribute__((address_space(1)))
#else
#define GG_DP
#endif
// a host pointer into a CS field (host code is type-checked in the device pass too)
template <class D, class Q> inline void cs_set(D& dst, Q src) { dst = (D)src; }
struct Seg { uint32_t line, lo, hi, pad; };       // a run of row (X) / column (Y) `line`: positions [lo, hi]
// device-driven quantum loop (gg_coherent_run): current quantum, launch index
// of its step 0, run over, quantum-end arrivals, active / blocked tiles, least
// next start, quanta completed, quantum length
enum { QS_Q = 0, QS_START, QS_DONE, QS_ARRIVED, QS_ACTIVE, QS_BLOCKED, QS_MIN_NEXT, QS_COUNT, QS_QPS,
       QS_BWAIT, QS_BMAX, QS_REL, QS_N };   // barrier waits, their latest arrival, release (max + 1, or 0)
constexpr uint32_t kBarWait = 2;          // Tile::blocked of a tile waiting at a BARRIER record
// gap cycles before a record (a BARRIER record is taken at the tile's clock)
__device__ __forceinline__ uint64_t rec_gap(uint32_t meta)
{
  return meta == GG_META_BARRIER ? 0ull : (uint64_t)((meta & 0x7FFFFFFFu) >> 1);
}

constexpr uint32_t kInLds = 512;       // inbox / port batch entries ordered in LDS (more: global scratch)
constexpr uint32_t kRqLds = 512;       // directory request FIFO entries staged in LDS
constexpr uint32_t kChunks = 128;      // record chunks per tile step
constexpr uint32_t kChunk = 16;        // records per chunk
constexpr uint32_t kQMax = 128;        // largest max_list_size of a queue staged in LDS (wave ops: 2 per lane)
constexpr uint32_t kNetCtr = 7;        // router / link counters a walker accumulates per position
constexpr size_t kWalkLdsMax = 160 * 1024;
constexpr uint32_t kWalkPkBytes = 5 * 8 + 7 * 4;   // t, send, key, zl, queue t | idx, pos, dpos, nf/status, rank, queue rank, queue slot

struct CP {
  uint32_t T, K, L;                      // tiles, logical shards, owned tiles
  uint32_t s1, a1, s2, a2, log_line, pol1, pol2;
  uint32_t E, dassoc, log_dsets, log_slices, W, R, QC, IC;
  uint32_t bits_req, bits_data, bits_ifc, max_list, analytical, dram_qm, dram_qtype, dram_qaux;
  uint32_t net, nsx, nsy, mw, mh, qimg;  // network model; X / Y segments; mesh; bytes of a queue image
  uint32_t msg_cap, seg_cap, walk_pk;    // pool records per parity; entries per segment list; walker LDS packets
  uint32_t seg_xcd;                      // > 0: runs interleaved by shard (seg_xcd shards), XCD-grouped walker blocks
  uint32_t cache_lds_off, cache_lds_bytes; // k_c_persist<true>: the tile's cache state in LDS after the step's
  uint32_t touch_each;                     // hit runs touch LRU rows one record at a time (> 16 ways; GG_COH_TOUCH_EACH=1)
  uint32_t walk_wide;                      // pipelined walkers take the one-wave sweep (the > 128-packet path; GG_COH_WALK_WIDE=1)
  uint32_t no_hit_runs;                    // 1: every record through app_access (hit runs off; 0 in the build)
  uint32_t mt1, mt2, mt_log;               // miss-type tracking of the L1-D / L2 (cfg flags), log2 set capacity
  uint32_t fast;                           // k_c_step<true> (Tile's F): register queues only, no miss types
  uint32_t mosi;                           // pr_l1_pr_l2_dram_directory_mosi: k_c_step<false, 1> (Tile's PR = 1)
  uint32_t shl2;                           // pr_l1_sh_l2_msi / _mesi: k_c_step<false, 2 / 3> (Tile's PR = 2 / 3)
  uint32_t mesi;                           // pr_l1_sh_l2_mesi
  uint64_t lat_l1d, lat_l1t, lat_l2d, lat_l2t, lat_dir, gap_ps, dram_proc, dram_cost;
  NocParams np;
};

__device__ __forceinline__ uint32_t class_bits(const CP& P, uint32_t c) { return c == 1 ? P.bits_data : c == 2 ? P.bits_ifc : P.bits_req; }
__device__ __forceinline__ uint32_t msg_bits(const CP& P, uint32_t t) { return class_bits(P, len_class(t)); }

struct CS {
  GG_DP uint64_t* l1_tag; GG_DP uint8_t* l1_meta; GG_DP uint8_t* l1_rr;
  GG_DP uint64_t* l2_tag; GG_DP uint8_t* l2_meta; GG_DP uint8_t* l2_rr;
  GG_DP uint64_t* cc;                          // [L][2][12]
  GG_DP uint64_t* mtab;                        // [L][2][2^mt_log] address sets (line | E 1 I 2 F 4), ~0 empty; when tracking
  GG_DP unsigned long long* mtc;               // [L][2][GG_NUM_MISS_TYPES] when tracking
  GG_DP uint64_t* st;                          // [L][GG_NUM_TILE_STATS]
  GG_DP TileSt* ts;                            // [L] the tiles' step state (one 64-B line each)
  GG_DP DEnt* dir; GG_DP uint64_t* dsh;              // [L][E], [L][E][W]
  GG_DP DEnt* rep; GG_DP uint64_t* rsh;              // [L][R], [L][R][W]
  GG_DP CReq* rq;                              // [L][QC]
  // MOSI: the FIFO's other request fields, the entries' Random states (XOR
  // kRng0), the cached data list + length, the protocol event counters
  GG_DP CReqX* rqx;                            // [L][QC]
  GG_DP uint64_t* drng; GG_DP uint64_t* rrng;        // [L][E], [L][R]
  GG_DP uint64_t* cdl; GG_DP uint32_t* ncdl;         // [L][kCdl], [L]
  GG_DP uint64_t* ps;                          // [L][GG_NUM_PROTO_STATS]
  GG_DP HQueue* dq; GG_DP HNode* dnd;                // DRAM queue per tile
  GG_DP const uint32_t* gtile; GG_DP const int32_t* ltile; GG_DP const uint32_t* shard;   // local -> tile, tile -> local (-1), tile -> shard
  GG_DP const uint4* tinfo;                    // [L] {tile, X run, Y run, 0} of a local tile: one load, no chain
  GG_DP const uint64_t* addr; GG_DP const uint32_t* meta; GG_DP uint64_t* out;
  GG_DP gg_cmsg* pool0; GG_DP gg_cmsg* pool1; GG_DP uint32_t* npool;    // records of even / odd steps, alloc counters [2]
  GG_DP uint32_t* inb0; GG_DP uint32_t* inb1;       // inbox record lists [L][IC]
  GG_DP uint32_t* arv0; GG_DP uint32_t* arv1;       // hop-by-hop SELF lists [L][IC]
  GG_DP uint32_t* cnt4;                       // [L][4]: the lists' lengths {inbox even, odd, SELF even, odd}
  // segment (run) lists [n][seg_cap] of {record index | destination tile << 32} (the
  // destination rides with the index so a walker's hand-off lookups start with
  // the record loads), their counts [n]
  GG_DP uint64_t* xl; GG_DP uint32_t* nxl; GG_DP uint64_t* yl; GG_DP uint32_t* nyl;
  GG_DP const Seg* segx; GG_DP const Seg* segy;
  GG_DP const uint32_t* tseg;                  // [T][2]: X run, Y run of a tile (~0 if not owned)
  GG_DP gg_cmsg* bnd; GG_DP uint32_t* bnd_cnt;       // held for the quantum boundary
  GG_DP uint32_t* ring; GG_DP uint32_t* quiet;       // records sent per step (mod 4); quiet flag of the quantum
  GG_DP uint32_t* imp;                         // [2] held packets imported for the quantum of parity Q & 1
  GG_DP uint32_t* live;                        // [4] launch L & 3: step index + 1 of a step launch, 0 otherwise
  GG_DP uint64_t* qs;                          // device-driven run: QS_* below
  GG_DP uint64_t* ri; GG_DP uint32_t* err;
  GG_DP HQueue* nq; GG_DP HNode* nnd;                // router queues [tile * 6 + port]
  GG_DP uint64_t* ctr;                         // NoC counters [T][GG_NUM_NET_COUNTERS]
  GG_DP uint64_t* gscr;                        // [L][6 * IC] ordering scratch beyond kInLds
  GG_DP unsigned long long* prof;              // GG_COH_PROFILE=1: shader-clock cycles per phase (diagnostics)
  // GG_COH_TRACE=n: per launch L < n, plain stores of every tile's / walker
  // block's phase clocks (trs [L][owned tile][16], trw [L][stage][block][8]);
  // no atomics, so the run's timing is barely disturbed (diagnostics)
  GG_DP unsigned long long* trs; GG_DP unsigned long long* trw; uint32_t tr_n, tr_wb;
  // GG_COH_TRACE_EV=n: walker events of launches [kTrEv0, kTrEv0 + n): per block
  // 128 x {memtime at the serve decision, after the request, after the
  // publish, packet | position << 16 | wave << 24 | poll count << 32} and a count
  GG_DP unsigned long long* tre; uint32_t tre_n;
  GG_DP uint32_t* gbar;                        // grid barrier counter of k_c_persist
  // in-kernel launch timing (gg_set_timing mode 2): per timed launch slot
  // {first workgroup start, last workgroup end} on the s_memrealtime clock
  GG_DP unsigned long long* kt; uint32_t kt_slot, kt_stride;   // timing mode 2: per block {start, end} of launch slot kt_slot
};
// profile slots: step phases 0..5 summed over tiles, 8 = sum over steps of the slowest tile;
// walker: 16 staging+load, 17 event loop, 18 hand-off+write back, 19 events, 20 sum of slowest walker per launch (X),
// 21 (Y), 22 launches
constexpr uint32_t kTrStep = 32;       // GG_COH_TRACE words per (launch, tile)
constexpr uint32_t kTrEv0 = 200, kTrEvMax = 128;
#define PROF_T0() const uint64_t _p0 = (DG(S.prof) || DG(S.trs)) ? __builtin_amdgcn_s_memtime() : 0
#define PROF_AT(var) const uint64_t var = (DG(S.prof) || DG(S.trs)) ? __builtin_amdgcn_s_memtime() : 0
// GG_COH_PROFILE batch shapes: per port kind (0 SELF, 1 injection, 2 walker),
// requests by batch size bucket (1, 2-3, 4-7, ..., 64+), requests at or after
// the last interval's start at the batch's start (a tail run)
__device__ __forceinline__ void prof_batch(const CS& S, int kind, uint32_t m, uint32_t tail)
{
  const int b = m <= 1 ? 0 : m <= 3 ? 1 : m <= 7 ? 2 : m <= 15 ? 3 : m <= 31 ? 4 : m <= 63 ? 5 : 6;
  atomicAdd(&DG(S.prof)[50 + 8 * kind + b], (unsigned long long)m);
  atomicAdd(&DG(S.prof)[80 + kind], (unsigned long long)tail);
}

__device__ __forceinline__ gg_cmsg* pool(const CS& S, uint32_t p) { return p ? S.pool1 : S.pool0; }
__device__ __forceinline__ uint32_t* inb(const CS& S, uint32_t p) { return p ? S.inb1 : S.inb0; }
__device__ __forceinline__ uint32_t* ninb_at(const CS& S, uint32_t p, size_t l) { return S.cnt4 + l * 4 + p; }
__device__ __forceinline__ uint32_t* arv(const CS& S, uint32_t p) { return p ? S.arv1 : S.arv0; }
__device__ __forceinline__ uint32_t* narv_at(const CS& S, uint32_t p, size_t l) { return S.cnt4 + l * 4 + 2 + p; }

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) { return (uint64_t)__shfl((long long)v, src); }
// lane l's value for a wave-uniform l (v_readlane, no LDS permute)
__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
// wave reductions on the VALU (DPP row shifts, then the row broadcasts; the
// result read from lane 63 is uniform): no LDS permutes, whose dependent
// chain of six costs ~300 cycles.  Called by the whole wave.
template <class Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v, uint32_t id, Op op)
{
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
  return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(v, 0u, [](uint32_t a, uint32_t b) { return a + b; }), 63);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(v, ~0u, [](uint32_t a, uint32_t b) { return a < b ? a : b; }), 63);
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t)
{
  return wave_scan_dpp(v, 0u, [](uint32_t a, uint32_t b) { return a + b; }) - v;
}
// pick the element of a per-thread register array selected by a lane-varying index
template <int N> __device__ __forceinline__ uint64_t pick(const uint64_t (&a)[N], uint32_t i)
{
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) if (i == (uint32_t)k) v = a[k];
  return v;
}
template <int N> __device__ __forceinline__ uint32_t pick(const uint32_t (&a)[N], uint32_t i)
{
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) if (i == (uint32_t)k) v = a[k];
  return v;
}

// ---------------------------------------------------------------------------
// one private cache (Cache + CacheSet + replacement policy, cache.cc / cache_set.cc):
// lane w handles way w of the set an operation touches
// ---------------------------------------------------------------------------
// a set's row of meta bytes (way i in byte i % 8 of half i / 8), <= 16 ways
__device__ __forceinline__ void load_row(const uint8_t* mr, uint32_t ways, uint64_t& ra, uint64_t& rb)
{
  if (ways == 4) { ra = *reinterpret_cast<const uint32_t*>(mr); rb = 0; }
  else if (ways == 8) { ra = *reinterpret_cast<const uint64_t*>(mr); rb = 0; }
  else if (ways == 16) { ra = reinterpret_cast<const uint64_t*>(mr)[0]; rb = reinterpret_cast<const uint64_t*>(mr)[1]; }
  else {
    ra = rb = 0;
    for (uint32_t w = 0; w < ways; ++w) { const uint64_t v = (uint64_t)mr[w] << (8 * (w & 7)); if (w < 8) ra |= v; else rb |= v; }
  }
}
__device__ __forceinline__ uint32_t row_byte(uint64_t ra, uint64_t rb, uint32_t w) { return (uint32_t)((w < 8 ? ra : rb) >> (8 * (w & 7))) & 0xFFu; }
// one record lane's share of a run's LRU row update (see l1_hit_run): the last
// touch of a way writes its age (distinct ways touched after it), the set's
// last record writes the untouched ways (a_i + #{touched t: a_t > a_i})
__device__ __forceinline__ void lru_run_store(uint8_t* mr, uint32_t ways, uint64_t ra, uint64_t rb, uint32_t w, uint32_t tm, uint32_t af)
{
  if (!((af >> w) & 1)) mr[w] = (uint8_t)((row_byte(ra, rb, w) & 7u) | ((uint32_t)__builtin_popcount(af) << 3));
  if (af) return;
  uint32_t am = 0;                                                   // ages of the touched ways
  for (uint32_t i = 0; i < ways; ++i) if ((tm >> i) & 1) am |= 1u << (row_byte(ra, rb, i) >> 3);
  for (uint32_t i = 0; i < ways; ++i) {
    if ((tm >> i) & 1) continue;
    const uint32_t b = row_byte(ra, rb, i), ai = b >> 3;
    mr[i] = (uint8_t)((b & 7u) | ((ai + (uint32_t)__builtin_popcount(am >> (ai + 1))) << 3));
  }
}
// inclusive prefix sum over the wave (DPP row shifts, then the row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v)
{
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return v;
}

template <bool MT>
struct CacheT {
  uint64_t* tag; uint8_t* meta; uint8_t* rr; uint64_t* cg;
  uint32_t sets, ways, log_line, pol, wb, ln;
  uint32_t cd;                         // this step's counter increments: lane k holds counter k
  // the last set this lane loaded (its way), kept in step with every store, so
  // consecutive operations on one set load it once
  uint32_t cset; uint64_t ctv; uint32_t cmv;
  // miss-type tracking (track_miss_types, cache.cc:321-405): the evicted /
  // invalidated / fetched address sets as one open-addressing table owned by
  // the tile (line address | bits), probed 64 slots per wave load
  uint64_t* mtab = nullptr; unsigned long long* mtc = nullptr; uint32_t mt_log = 0;
  uint32_t e3 = 0;                     // state code 3 is MESI's EXCLUSIVE (clean), not MOSI's OWNED
  static constexpr uint64_t kMtEmpty = ~0ull;
  static constexpr uint32_t kMtE = 1, kMtI = 2, kMtF = 4;
  __device__ __forceinline__ uint64_t mt_slot(uint64_t a, uint32_t& bits, uint32_t& err)
  {
    const uint64_t cap = 1ull << mt_log;
    uint64_t h = (a >> log_line) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    for (uint64_t base = h & (cap - 1), n = 0; n < cap; base = (base + 64) & (cap - 1), n += 64) {
      const uint64_t i = (base + ln) & (cap - 1);
      const uint64_t k = mtab[i];
      const uint64_t hit = __ballot(k != kMtEmpty && (k & ~7ull) == a), emp = __ballot(k == kMtEmpty);
      const uint64_t any = hit | emp;                                  // probe order = lane order
      if (any) {
        const uint32_t l = (uint32_t)__builtin_ctzll(any);
        bits = (hit >> l) & 1 ? (uint32_t)(rl64(k, l) & 7u) : 0u;
        return (base + l) & (cap - 1);
      }
    }
    err |= GG_DERR_CAP;                                                // the table is full (miss_track_lines)
    bits = 0;
    return ~0ull;
  }
  __device__ __forceinline__ void mt_put(uint64_t i, uint64_t a, uint32_t bits)
  {
    if (i == ~0ull) return;                                            // full: the run is flagged, no slot is overwritten
    if (ln == 0) mtab[i] = a | bits;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __device__ __forceinline__ void mt_or(uint64_t a, uint32_t b, uint32_t& err)
  {
    uint32_t bits;
    const uint64_t i = mt_slot(a, bits, err);
    mt_put(i, a, bits | b);
  }
  // insertCacheLine (cache.cc:131-148): the victim into the evicted set; the
  // inserted line out of the first set that holds it (clearMissTypeTrackingSets,
  // :398-404), then into the fetched set
  __device__ __forceinline__ void mt_insert(uint64_t a, bool ev, uint64_t ev_addr, uint32_t& err)
  {
    if (ev) mt_or(ev_addr, kMtE, err);
    uint32_t bits;
    const uint64_t i = mt_slot(a, bits, err);
    if (bits & kMtE) bits &= ~kMtE;
    else if (bits & kMtI) bits &= ~kMtI;
    else if (bits & kMtF) bits &= ~kMtF;
    mt_put(i, a, bits | kMtF);
  }
  // getMissType + updateMissTypeCounters (cache.cc:363-396)
  __device__ __forceinline__ void mt_classify(uint64_t a, uint32_t& err)
  {
    uint32_t bits;
    (void)mt_slot(a, bits, err);
    const uint32_t t = (bits & kMtE) ? GG_MT_CAPACITY : (bits & (kMtI | kMtF)) ? GG_MT_SHARING : GG_MT_COLD;
    if (ln == 0) atomicAdd(&mtc[t], 1ull);
  }
  uint32_t mt_err = 0;

  __device__ __forceinline__ void cnt(uint32_t k) { if (ln == k) ++cd; }
  __device__ __forceinline__ void cnt_add(uint32_t k, uint32_t v) { if (ln == k) cd += v; }
  __device__ __forceinline__ uint32_t set_of(uint64_t a) const { return (uint32_t)((a >> log_line) & (sets - 1)); }   // cache_hash_fn.h:17
  __device__ __forceinline__ uint64_t tag_of(uint64_t a) const { return a >> log_line; }                             // cache.cc:495
  __device__ __forceinline__ void ld(uint32_t s, uint64_t& tv, uint32_t& mv)
  {
    if (s != cset) {
      ctv = INV_ADDR; cmv = 0;
      if (ln < ways) { ctv = tag[(size_t)s * ways + ln]; cmv = meta[(size_t)s * ways + ln]; }
      cset = s;
    }
    tv = ctv; mv = cmv;
  }
  __device__ __forceinline__ void st_meta(uint32_t s, uint32_t v)      // this lane's way
  {
    meta[(size_t)s * ways + ln] = (uint8_t)v;
    if (s == cset) cmv = v;
  }
  __device__ __forceinline__ void st_tag(uint32_t s, uint64_t v)
  {
    tag[(size_t)s * ways + ln] = v;
    if (s == cset) ctv = v;
  }
  // CacheSet::find (cache_set.cc:57-70): tags are unique, so any matching lane is the way
  __device__ __forceinline__ int way_of(uint64_t tv, uint64_t t) const
  {
    const uint64_t m = __ballot(ln < ways && tv == t);
    return m ? (int)__builtin_ctzll(m) : -1;
  }
  __device__ __forceinline__ void touch(uint32_t s, int w, uint32_t mv)                                           // lru:40-50
  {
    if (pol != GG_POLICY_LRU) return;
    const uint32_t acc = rl32(mv, (uint32_t)w) >> 3;
    if (ln < ways) {
      const uint32_t a = mv >> 3;
      uint32_t nv = mv;
      if ((int)ln == w) nv = mv & 7u;
      else if (a < acc) nv = (mv & 7u) | ((a + 1) << 3);
      if (nv != mv) st_meta(s, nv);
    }
  }
  __device__ __forceinline__ void miss_counters(uint64_t a, bool wr, bool miss)                                   // cache.cc:321-360
  {
    cnt(GG_CC_ACCESSES);
    if (wr) cnt(GG_CC_WRITE_ACCESSES); else cnt(GG_CC_READ_ACCESSES);
    if (miss) {
      cnt(GG_CC_MISSES); if (wr) cnt(GG_CC_WRITE_MISSES); else cnt(GG_CC_READ_MISSES);
      if (MT && mtab) mt_classify(a, mt_err);
    }
  }
  // getCacheLineInfo (cache.cc:187-215): state / loc of the line, I / 0 when absent
  __device__ __forceinline__ void get(uint64_t a, uint32_t& st, uint32_t& loc)
  {
    uint64_t tv; uint32_t mv;
    ld(set_of(a), tv, mv);
    const int w = way_of(tv, tag_of(a));
    cnt(GG_CC_TAG_READS);
    if (w >= 0) { const uint32_t m = rl32(mv, (uint32_t)w); st = m & 3u; loc = (m >> 2) & 1u; }
    else { st = ST_I; loc = 0; }
  }
  // the line's state without the TAG_READ count (hit-run predictor)
  __device__ __forceinline__ uint32_t probe(uint64_t a)
  {
    uint64_t tv; uint32_t mv;
    ld(set_of(a), tv, mv);
    const int w = way_of(tv, tag_of(a));
    return w >= 0 ? rl32(mv, (uint32_t)w) & 3u : (uint32_t)ST_I;
  }
  // setCacheLineInfo (cache.cc:218-241): st == I writes the invalid tag (CacheLineInfo::invalidate)
  __device__ __forceinline__ bool set(uint64_t a, uint32_t st, uint32_t loc)
  {
    const uint32_t s = set_of(a);
    uint64_t tv; uint32_t mv;
    ld(s, tv, mv);
    const int w = way_of(tv, tag_of(a));
    if (w < 0) return false;
    if (MT && mtab && st == ST_I) mt_or(a, kMtI, mt_err);                  // cache.cc:228-230
    if ((int)ln == w) {
      st_meta(s, (mv & 0xF8u) | st | (loc << 2));
      if (st == ST_I) st_tag(s, INV_ADDR);
    }
    cnt(GG_CC_TAG_WRITES);
    return true;
  }
  // accessCacheLine (cache.cc:84-112)
  __device__ __forceinline__ bool access(uint64_t a, bool store)
  {
    const uint32_t s = set_of(a);
    uint64_t tv; uint32_t mv;
    ld(s, tv, mv);
    const int w = way_of(tv, tag_of(a));
    if (w < 0) return false;
    touch(s, w, mv);
    if (store) cnt(GG_CC_DATA_WRITES); else cnt(GG_CC_DATA_READS);
    return true;
  }
  // insertCacheLine (cache.cc:114-184) with getReplacementWay: LRU (lru:23-38) = first
  // invalid way, else the way of age assoc-1; round robin (rr:13-22)
  __device__ __forceinline__ bool insert(uint64_t a, uint32_t st, uint32_t loc, bool& ev, uint64_t& ev_addr,
                                         uint32_t& ev_st, uint32_t& ev_loc)
  {
    const uint32_t s = set_of(a);
    uint64_t tv; uint32_t mv;
    ld(s, tv, mv);
    int w;
    if (pol == GG_POLICY_LRU) {
      const uint64_t inv = __ballot(ln < ways && tv == INV_ADDR);
      const uint64_t old = __ballot(ln < ways && tv != INV_ADDR && (mv >> 3) == ways - 1);
      w = inv ? (int)__builtin_ctzll(inv) : (old ? (int)__builtin_ctzll(old) : -1);
    } else {
      const uint32_t cur = rr[s];
      rr[s] = (uint8_t)(cur == 0 ? ways - 1 : cur - 1);
      w = (int)cur;
    }
    if (w < 0 || (uint32_t)w >= ways) return false;
    const uint64_t vt = rl64(tv, (uint32_t)w);
    const uint32_t vm = rl32(mv, (uint32_t)w);
    ev = vt != INV_ADDR;
    if (ev) { ev_addr = vt << log_line; ev_st = vm & 3u; ev_loc = (vm >> 2) & 1u; }
    if (MT && mtab) mt_insert(a, ev, vt << log_line, mt_err);
    if ((int)ln == w) {
      const uint32_t nm = (vm & 0xF8u) | st | (loc << 2);
      st_tag(s, tag_of(a));
      st_meta(s, nm);
      mv = nm;
    }
    touch(s, w, mv);
    cnt(GG_CC_TAG_READS);
    if (ev) {
      cnt(GG_CC_DATA_READS);
      cnt(GG_CC_EVICTIONS);
      if (wb && (ev_st == ST_M || (ev_st == ST_O && !e3))) cnt(GG_CC_DIRTY_EVICTIONS);   // CacheState::dirty(): M / O
    }
    cnt(GG_CC_TAG_WRITES); cnt(GG_CC_DATA_WRITES);
    return true;
  }
};

// work items of the directory controller's call chains (recursion in the
// reference, an explicit continuation stack here)
enum { W_NONE = 0, W_PROC, W_CONT, W_NEXT, W_NULLIFY };
struct Work { uint64_t addr; uint32_t kind, type, requester, cached; int32_t h; };
#define WSTACK 32

// LDS of one tile step (IN: inbox / port batch entries ordered in LDS, RQ:
// directory request FIFO entries staged in LDS; beyond them global scratch)
template <uint32_t IN, uint32_t RQ>
struct StepLdsT {
  static constexpr uint32_t kIn = IN, kRq = RQ;
  CReq rq[RQ];
  uint8_t dimg[sizeof(HQueue) + kQMax * sizeof(HNode)];   // DRAM queue image
  uint8_t pimg[sizeof(HQueue) + kQMax * sizeof(HNode)];   // SELF / injection port image
  uint64_t x1[IN], x2[IN], x3[IN], x4[IN];
  uint32_t i1[IN], i2[IN];
  uint32_t ch[2 * kChunks];                               // record chunks: base, used
  Work wstack[WSTACK];                                    // directory work loop continuations
};
using StepLds = StepLdsT<kInLds, kRqLds>;                 // one tile per workgroup (k_c_step, k_c_persist)

// The lanes of ONE wave exchange data through LDS / global memory between the
// phases of a tile step; in a multi-wave workgroup the other waves run other
// tiles, so this is a wave barrier with workgroup-scope fences (every wait a
// __syncthreads would imply, no s_barrier).  With one wave per workgroup
// (k_c_step, k_c_persist) the compiler emits these as wavefront-scope: no
// wait for outstanding global accesses.
__device__ __forceinline__ void tsync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Where a tile step's deliveries go.  GHooks: the per-step launches
// (k_c_step / k_c_persist) keep the inbox / arrival / segment counters and the
// record pools in HBM, shared by every block of the launch.  Slot functions
// return the list position or ~0u (capacity exceeded, reported through S.err).
struct GHooks {
  const CP& P; const CS& S;
  // n contiguous records of the parity-p pool (wave-uniform)
  __device__ __forceinline__ uint32_t pool_alloc(uint32_t p, uint32_t want) const
  {
    uint32_t b = 0;
    if (lane_id() == 0) b = atomicAdd(&(p ? S.npool[1] : S.npool[0]), want);
    b = (uint32_t)__shfl((int)b, 0);
    return (uint64_t)b + want > P.msg_cap ? ~0u : b;
  }
  __device__ __forceinline__ uint32_t inbox_slot(uint32_t pn, uint32_t ld) const
  {
    const uint32_t j = atomicAdd(ninb_at(S, pn, ld), 1u);
    return j < P.IC ? j : ~0u;
  }
  __device__ __forceinline__ uint32_t arv_slot(uint32_t pn, uint32_t ld) const
  {
    const uint32_t j = atomicAdd(narv_at(S, pn, ld), 1u);
    return j < P.IC ? j : ~0u;
  }
  __device__ __forceinline__ uint32_t seg_slot(bool is_x, uint32_t sg) const
  {
    const uint32_t j = atomicAdd(&(is_x ? S.nxl : S.nyl)[sg], 1u);
    return j < P.seg_cap ? j : ~0u;
  }
  __device__ __forceinline__ bool bnd_put(const gg_cmsg& m) const
  {
    const uint32_t j = atomicAdd(S.bnd_cnt, 1u);
    if (j >= P.msg_cap) return false;
    S.bnd[j] = m;
    return true;
  }
  // the tile's delivery counts of parity p were consumed
  __device__ __forceinline__ void clear_arv(uint32_t p, uint32_t lt) const { *narv_at(S, p, lt) = 0; }
  __device__ __forceinline__ void clear_inb(uint32_t p, uint32_t lt) const { *ninb_at(S, p, lt) = 0; }
  // lane 0: the step's run-info counts
  __device__ __forceinline__ void step_counts(uint32_t k, uint32_t net, uint32_t self, uint32_t bnd, uint32_t sent) const
  {
    if (net) atomicAdd((unsigned long long*)&S.ri[GG_RI_NET_MSGS], (unsigned long long)net);
    if (self) atomicAdd((unsigned long long*)&S.ri[GG_RI_SELF_MSGS], (unsigned long long)self);
    if (bnd) atomicAdd((unsigned long long*)&S.ri[GG_RI_BOUNDARY_MSGS], (unsigned long long)bnd);
    if (sent) atomicAdd(&S.ring[k & 3], sent);
  }
};

// the tile's per-step state words, loaded at kernel entry together with the
// launch state (one memory round trip instead of a chain behind it)
struct TilePre {
  uint32_t tile;
  uint64_t rec, rec_end, clk, pend_start, out_addr, out_time;
  uint32_t blocked, seq, nrep, nrq;
  uint64_t ccv, stv;
  uint32_t narv0, narv1, ninb0, ninb1;   // both parities (scalars: no dynamically indexed private array)
  uint32_t segx, segy;                   // the tile's X / Y run (hop-by-hop), ~0 otherwise
  __device__ __forceinline__ void load(const CS& S, uint32_t lt, uint32_t ln)
  {
    const uint4 ti = S.tinfo[lt];
    tile = ti.x; segx = ti.y; segy = ti.z;
    rec = S.ts[lt].rec; rec_end = S.ts[lt].rec_end; clk = S.ts[lt].clk; pend_start = S.ts[lt].pend_start;
    out_addr = S.ts[lt].out_addr; out_time = S.ts[lt].out_time;
    blocked = S.ts[lt].blocked; seq = S.ts[lt].seq; nrep = S.ts[lt].nrep; nrq = S.ts[lt].nrq;
    ccv = ln < 2 * GG_NUM_CACHE_COUNTERS ? S.cc[(size_t)lt * 2 * GG_NUM_CACHE_COUNTERS + ln] : 0;
    stv = ln < GG_NUM_TILE_STATS ? S.st[(size_t)lt * GG_NUM_TILE_STATS + ln] : 0;
    const uint4 c = reinterpret_cast<const uint4*>(S.cnt4)[lt];      // one 16-B load
    ninb0 = c.x; ninb1 = c.y; narv0 = c.z; narv1 = c.w;
  }
};

// ---------------------------------------------------------------------------
// one tile's controllers (every lane, identical values)
// ---------------------------------------------------------------------------
// F: the fast instance (k_c_step<true>, chosen on the host by coh_fast):
// every queue a step serves — the router ports and the DRAM queue — is a
// history tree of <= kQMax intervals held in registers (RegQueue), and no
// cache tracks miss types, so the other queue forms and the miss-type hooks
// are compiled out of it (a smaller kernel: fewer instruction-cache misses
// on a tile's path, fewer live values)
// MO: the MOSI controllers (pr_l1_pr_l2_dram_directory_mosi, k_c_step<false,
// true>): OWNED lines and entries, upgrade replies, combined invalidate-flush
// requests, sharer write-backs, the directory's cached data list and the
// protocol event counters (directory_msg_mo / l2_msg_mo below)
// PR: the caching protocol — 0 pr_l1_pr_l2_dram_directory_msi, 1 its MOSI
// form (MO), 2 pr_l1_sh_l2_msi (SH: the L2 a shared slice per tile whose lines
// carry the directory entries, sh_* below), 3 pr_l1_sh_l2_mesi (SH and ME:
// EXCLUSIVE L1 lines)
template <class SL, class H, bool F = false, int PR = 0>
struct Tile {
  static constexpr bool MO = PR == 1, SH = PR >= 2, ME = PR == 3;
  static constexpr bool kF = F;
  static constexpr bool kMO = MO;
  using Cache = CacheT<!F>;
  const CP& P; const CS& S;
  uint32_t lt, tile, ln, p;             // local index, tile id, lane, step parity
  SL& sl;
  const H& hk;
  Cache L1, L2;
  uint64_t sd;                          // this step's statistics increments: lane k holds statistic k
  uint64_t rec, rec_end, clk, pend_start, out_addr, out_time;
  uint32_t blocked, seq, nrep, nrq;
  bool dq_lds;                          // the DRAM queue image in LDS (sl.dimg), else in HBM
  GG_GLB CReq* rqg; bool rq_lds;         // the request FIFO in HBM, or in LDS (sl.rq) when it fits
  uint32_t nch, cbase, cused, ccap, nsent;
  bool failed;
  uint32_t ferr;                         // GG_DERR_* gathered by fail()
  uint32_t fline = 0;                    // the source line of the first fail()
  uint64_t ccv, stv;                    // lane k's cache counter k (of 2 x 12) and statistic k, loaded at step start
  const TilePre& p0;                    // the state loaded at step start (flush stores only what changed)
  int32_t oh = NO_ENT; bool od = false;  // the open directory entry (eopen) and whether it changed
  uint64_t oaddr = 0, osh = 0; int32_t oown = -1; uint32_t ost = 0, onsh = 0;
  bool tr_on = false;                   // GG_COH_TRACE: cycles by handler part (dget, sharers, DRAM, send, FIFO, sharer words)
  uint64_t tra[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // + directory_msg before the run, the run, entry opens
  // MOSI: event counter increments (lane k holds counter k), the cached data
  // list's length (and at step start), the FIFO's MOSI fields
  uint64_t pd = 0;
  uint32_t ncdl = 0, ncdl0 = 0;
  GG_GLB CReqX* rqx = nullptr;
  // the directory's per-tile arrays and sharer words per entry, formed once
  // per step: ent / shw run on every handler's path, and formed there from
  // CP / CS each call re-read those fields with scalar loads and waited
  GG_DP DEnt* dirb; GG_DP DEnt* repb;
  GG_DP uint64_t* dshb; GG_DP uint64_t* rshb;
  uint32_t wd;
  GG_DP gg_cmsg* cpool;                 // this step's record pool (put)

  // LC: the tile's L1-D / L2 tags, meta bytes and RR counters live in LDS at
  // clds for the whole launch (k_c_persist; layout of cache_lds_bytes)
  template <bool LC>
  __device__ __forceinline__ Tile(const CP& P_, const CS& S_, uint32_t l, uint32_t par, SL& s_, const H& h_, uint8_t* clds,
                                  std::integral_constant<bool, LC>, const TilePre& pre)
      : P(P_), S(S_), lt(l), tile(pre.tile), ln(lane_id()), p(par), sl(s_), hk(h_), p0(pre)
  {
    const size_t n1 = (size_t)P.s1 * P.a1, n2 = (size_t)P.s2 * P.a2;
    if constexpr (LC) {
      uint64_t* t1 = reinterpret_cast<uint64_t*>(clds);
      uint64_t* t2 = t1 + n1;
      uint8_t* m1 = reinterpret_cast<uint8_t*>(t2 + n2);
      uint8_t* m2 = m1 + n1;
      uint8_t* r1 = m2 + n2;
      uint8_t* r2 = r1 + P.s1;
      L1 = Cache{t1, m1, r1, S.cc + (size_t)lt * 2 * GG_NUM_CACHE_COUNTERS, P.s1, P.a1, P.log_line, P.pol1, 0, ln, 0, ~0u, 0, 0};
      L2 = Cache{t2, m2, r2, S.cc + ((size_t)lt * 2 + 1) * GG_NUM_CACHE_COUNTERS, P.s2, P.a2, P.log_line, P.pol2, 1, ln, 0,
                 ~0u, 0, 0};
    } else {
      // the L1-D is write-through under pr_l1_pr_l2 (l1_cache_cntlr.cc:59), write-back under sh_l2 (…sh_l2_msi/l1:57)
      L1 = Cache{S.l1_tag + lt * n1, S.l1_meta + lt * n1, S.l1_rr + (size_t)lt * P.s1,
                 S.cc + (size_t)lt * 2 * GG_NUM_CACHE_COUNTERS, P.s1, P.a1, P.log_line, P.pol1, SH ? 1u : 0u, ln, 0, ~0u, 0, 0};
      L2 = Cache{S.l2_tag + lt * n2, S.l2_meta + lt * n2, S.l2_rr + (size_t)lt * P.s2,
                 S.cc + ((size_t)lt * 2 + 1) * GG_NUM_CACHE_COUNTERS, P.s2, P.a2, P.log_line, P.pol2, 1, ln, 0, ~0u, 0, 0};
    }
    if constexpr (ME) L1.e3 = 1;
    if (!F && P.mt1) {
      L1.mtab = S.mtab + ((size_t)lt * 2 << P.mt_log); L1.mtc = S.mtc + (size_t)lt * 2 * GG_NUM_MISS_TYPES;
      L1.mt_log = P.mt_log;
    }
    if (!F && P.mt2) {
      L2.mtab = S.mtab + (((size_t)lt * 2 + 1) << P.mt_log); L2.mtc = S.mtc + ((size_t)lt * 2 + 1) * GG_NUM_MISS_TYPES;
      L2.mt_log = P.mt_log;
    }
    sd = 0;
    dirb = S.dir + (size_t)lt * P.E; repb = S.rep + (size_t)lt * P.R;
    dshb = S.dsh + (size_t)lt * P.E * P.W; rshb = S.rsh + (size_t)lt * P.R * P.W; wd = P.W;
    cpool = p ? S.pool1 : S.pool0;
    rec = pre.rec; rec_end = pre.rec_end; clk = pre.clk; pend_start = pre.pend_start;
    out_addr = pre.out_addr; out_time = pre.out_time;
    blocked = pre.blocked; seq = pre.seq; nrep = pre.nrep; nrq = pre.nrq;
    dq_lds = false;
    rqg = (GG_GLB CReq*)(S.rq + (size_t)lt * P.QC); rq_lds = false;
    nch = 0; cbase = 0; cused = 0; ccap = 0; nsent = 0; failed = false; ferr = 0;
    ccv = pre.ccv; stv = pre.stv;
    if constexpr (MO) {
      rqx = (GG_GLB CReqX*)(S.rqx + (size_t)lt * P.QC);
      ncdl = ncdl0 = S.ncdl[lt];
    }
  }
  __device__ __forceinline__ void stat(uint32_t k, uint64_t v) { if (ln == k) sd += v; }
  __device__ __forceinline__ void pstat(uint32_t k, uint64_t v = 1) { if (ln == k) pd += v; }   // MOSI event counters
  // error flags are gathered in a register and reported once per step
  // (flush_err): one atomic site instead of one per inlined check
  // (line: the call site's line in this file, reported with the first failure)
  __device__ __forceinline__ void fail(uint32_t e = GG_DERR_STATE, uint32_t line = __builtin_LINE())
  {
    if (!failed) fline = line;
    failed = true;
    ferr |= e;
  }
  __device__ __forceinline__ void flush_err()
  {
    ferr |= L1.mt_err | L2.mt_err;
    if (ferr && ln == 0) { atomicOr(S.err, ferr); if (fline) atomicCAS(S.err + 1, 0u, fline); }
  }

  // ---- records (MemoryManager::sendMsg, …msi/memory_manager.cc:306-332) ------
  // n contiguous record slots of this step's pool, from the tile's current chunk
  __device__ __forceinline__ uint32_t alloc(uint32_t n)
  {
    if (failed) return ~0u;
    if (cused + n > ccap) {
      if (nch) sl.ch[2 * (nch - 1) + 1] = cused;
      const uint32_t want = n > kChunk ? n : kChunk;
      // the tile's first chunk of a step is its own slice of the pool (no
      // atomic on the critical path); later ones come from the shared part
      // above the P.L slices (the pool counters start there)
      const uint32_t b = nch == 0 && want == kChunk ? lt * kChunk : hk.pool_alloc(p, want);
      if (b == ~0u || nch >= kChunks) { fail(GG_DERR_CAP); return ~0u; }
      sl.ch[2 * nch] = b; sl.ch[2 * nch + 1] = 0;
      ++nch; cbase = b; ccap = want; cused = 0;
    }
    const uint32_t i = cbase + cused;
    cused += n; nsent += n;
    return i;
  }
  __device__ __forceinline__ void put(uint32_t i, uint32_t dst, uint32_t type, uint32_t requester, uint64_t addr,
                                      uint64_t t, uint32_t sq, uint32_t single_rx = 0)
  {
    gg_cmsg m;
    m.addr = addr; m.send_ps = t; m.arrival_ps = t; m.zero_load_ps = 0;
    m.src = tile; m.dst = dst; m.requester = requester; m.seq = sq; m.type = type; m.link = 0;
    m.hop = GG_HOP_NONE; m.single_rx = single_rx;
    cpool[i] = m;
    // the step's sent list in LDS (slot = send order = sq - the step's first
    // seq): publish reads its records' fields from here, not back from HBM
    // (x3 / x4 are free once the inbox is ordered; sends come after that)
    const uint32_t slot = sq - p0.seq;
    if (slot < SL::kIn) {
      sl.x3[slot] = (uint64_t)i | ((uint64_t)dst << 32) | ((uint64_t)len_class(type) << 62);   // dst < 2^30
      sl.x4[slot] = t;
    }
  }
  __device__ __forceinline__ void count_sent(uint32_t type, uint64_t n)
  {
    stat(GG_CT_MSGS_SENT, n);
    if (type - 1u < 11u) stat(GG_CT_SENT_BY_TYPE + type - 1u, n);
    else if (MO && type == M_IFC_REQ) stat(GG_CT_SENT_INV_FLUSH_COMBINED, n);
    else if (SH && type >= M_DRAM_FETCH_REQ && type <= M_DRAM_FETCH_REP) stat(GG_CT_SENT_DRAM_FETCH_REQ + type - M_DRAM_FETCH_REQ, n);
  }
  __device__ __forceinline__ void send(uint32_t dst, uint32_t type, uint32_t requester, uint64_t addr, uint64_t t)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; send_(dst, type, requester, addr, t); if (tr_on) tra[3] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void send_(uint32_t dst, uint32_t type, uint32_t requester, uint64_t addr, uint64_t t)
  {
    const uint32_t i = alloc(1);
    if (i == ~0u) return;
    put(i, dst, type, requester, addr, t, seq++);
    count_sent(type, 1);
  }
  __device__ __forceinline__ uint32_t home(uint64_t a) const { return (uint32_t)((a >> 6) % P.T); }   // address_home_lookup.cc:19-26

  // ---- directory (DirectoryCache + DirectoryEntryFullMap) ------------------
  // (h is wave-uniform: readfirstlane keeps the entry / sharer-word pointers
  // scalar — a per-lane select between the two arrays would hold both bases
  // in VGPRs for the whole step; rep_ent serves the per-lane scans of the
  // replaced list)
  __device__ __forceinline__ DEnt* ent(int32_t h) const
  {
    h = __builtin_amdgcn_readfirstlane(h);
    return h >= 0 ? dirb + h : repb + (-h - 1);
  }
  __device__ __forceinline__ uint64_t* shw(int32_t h) const
  {
    h = __builtin_amdgcn_readfirstlane(h);
    return h >= 0 ? dshb + (size_t)h * wd : rshb + (size_t)(-h - 1) * wd;
  }
  __device__ __forceinline__ const DEnt* rep_ent(uint32_t i) const { return repb + i; }
  // The open entry: the directory entry the current message works on, its
  // fields in scalars and its sharer words in lanes 0..W-1 (W <= 64), so a
  // handler's read-modify-writes of the entry are register operations (in
  // HBM each load behind a store waits for that store: ~1 µs apiece).
  // Written back when another entry opens, before the directory moves
  // entries (dreplace / dinvalidate / the replacement scan) and at step end.
  __device__ __forceinline__ void eopen(int32_t h)
  {
    h = __builtin_amdgcn_readfirstlane(h);
    if (h == oh) return;
    const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0;
    eopen_(h);
    if (tr_on) tra[8] += __builtin_amdgcn_s_memtime() - c0;
  }
  __device__ __forceinline__ void eopen_(int32_t h)
  {
    eclose();
    const DEnt* e = ent(h);
    oaddr = e->addr; oown = e->owner; ost = e->dstate; onsh = e->nsh;
    osh = ln < wd ? shw(h)[ln] : 0ull;
    oh = h; od = false;
  }
  __device__ __forceinline__ void eflush()
  {
    if (oh == NO_ENT || !od) return;
    DEnt* e = ent(oh);
    e->owner = oown; e->dstate = (uint16_t)ost; e->nsh = (uint16_t)onsh;
    if (ln < wd) shw(oh)[ln] = osh;
    od = false;
  }
  __device__ __forceinline__ void eclose() { eflush(); oh = NO_ENT; }
  __device__ __forceinline__ uint32_t e_state(int32_t h) { eopen(h); return ost; }
  __device__ __forceinline__ int32_t e_owner(int32_t h) { eopen(h); return oown; }
  __device__ __forceinline__ uint32_t e_nsh(int32_t h) { eopen(h); return onsh; }
  __device__ __forceinline__ void set_state(int32_t h, uint32_t st) { eopen(h); ost = st; od = true; }
  __device__ __forceinline__ uint64_t e_word(int32_t h, uint32_t w)
  {
    eopen(h);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(osh >> 32), (int)w) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)osh, (int)w);
  }
  __device__ __forceinline__ bool has(int32_t h, uint32_t s) { return (e_word(h, s >> 6) >> (s & 63)) & 1ull; }
  __device__ __forceinline__ void add_sharer(int32_t h, uint32_t s)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; add_sharer_(h, s); if (tr_on) tra[5] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void add_sharer_(int32_t h, uint32_t s)                 // addSharer (full_map.cc:27-33)
  {
    if (has(h, s)) fail();
    if (ln == (s >> 6)) osh |= 1ull << (s & 63);
    ++onsh; od = true;
  }
  __device__ __forceinline__ void remove_sharer(int32_t h, uint32_t s)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; remove_sharer_(h, s); if (tr_on) tra[5] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void remove_sharer_(int32_t h, uint32_t s)              // removeSharer (:35-41)
  {
    if (!has(h, s)) { fail(); return; }
    if (ln == (s >> 6)) osh &= ~(1ull << (s & 63));
    --onsh; od = true;
  }
  __device__ __forceinline__ void set_owner(int32_t h, int32_t o)                   // DirectoryEntry::setOwner
  {
    if (o >= 0 && !has(h, (uint32_t)o)) fail();
    eopen(h);
    oown = o; od = true;
  }
  __device__ __forceinline__ uint32_t dset(uint64_t a) const                        // computeSetIndex (directory_cache.cc:332-348)
  {
    uint64_t s = 0;
    const uint64_t mask = (1ull << P.log_dsets) - 1;
    for (uint32_t i = P.log_line + P.log_slices; i + P.log_dsets <= 64; i += P.log_dsets) s ^= (a >> i) & mask;
    return (uint32_t)s;
  }
  // getDirectoryEntry (directory_cache.cc:102-145): lane i checks way i, then replaced entry i
  __device__ __forceinline__ int32_t dget(uint64_t a, uint64_t& t)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; const int32_t r_ = dget_(a, t); if (tr_on) tra[0] += __builtin_amdgcn_s_memtime() - c0; return r_; }
  __device__ __forceinline__ int32_t dget_(uint64_t a, uint64_t& t)
  {
    t += P.lat_dir;
    stat(GG_CT_DIR_ACCESSES, 1);
    const uint32_t base = dset(a) * P.dassoc;
    DEnt* d = dirb;
    // one round of loads: the set's entries (lane = way) and, when they fit
    // four words per lane, the set's sharer words (word idx = way * W + k in
    // lane idx & 63 of register idx >> 6): a hit opens its entry (eopen)
    // without a dependent load
    const bool spec = wd * P.dassoc <= 256 && (wd & (wd - 1)) == 0;   // (W a power of two: an entry's words never straddle two registers)
    DEnt e{INV_ADDR, -1, 0, 0};
    if (ln < P.dassoc) e = d[base + ln];
    uint64_t sw0 = 0, sw1 = 0, sw2 = 0, sw3 = 0;
    if (spec) {
      const uint64_t* g = dshb + (size_t)base * wd;
      const uint32_t nw = wd * P.dassoc;
      if (ln < nw) sw0 = g[ln];
      if (ln + 64 < nw) sw1 = g[ln + 64];
      if (ln + 128 < nw) sw2 = g[ln + 128];
      if (ln + 192 < nw) sw3 = g[ln + 192];
    }
    const uint64_t hit = __ballot(ln < P.dassoc && e.addr == a);
    if (hit) {
      const uint32_t w = (uint32_t)__builtin_ctzll(hit);
      const int32_t h = (int32_t)(base + w);
      if (spec && oh != h) {                       // an open entry is newer than HBM: keep it
        eclose();
        oaddr = a;
        oown = (int32_t)rl32((uint32_t)e.owner, w);
        ost = rl32((uint32_t)e.dstate, w);
        onsh = rl32((uint32_t)e.nsh, w);
        const uint32_t i0 = w * wd, u = i0 >> 6;                    // the entry's words: one register
        const uint64_t src = u == 0 ? sw0 : u == 1 ? sw1 : u == 2 ? sw2 : sw3;
        const uint64_t x = shfl64(src, (int)((i0 + ln) & 63));
        osh = ln < wd ? x : 0ull;
        oh = h; od = false;
      }
      return h;
    }
    const uint64_t fr = __ballot(ln < P.dassoc && e.addr == INV_ADDR);
    if (fr) {
      // a never-used slot: its sharer words are zeroed here, not at reset
      // (full-map vectors of every entry are 2 GB at 1024 tiles); opened
      // with its reset fields (owner -1, UNCACHED, no sharers)
      const uint32_t w = (uint32_t)__builtin_ctzll(fr);
      const uint32_t i = base + w;
      if (oh == (int32_t)i) eclose();
      d[i].addr = a;
      if (ln < wd) shw((int32_t)i)[ln] = 0;
      if constexpr (MO) S.drng[(size_t)lt * P.E + i] = 0;          // a fresh Random (seed state)
      if (spec) {
        eclose();
        oaddr = a; oown = (int32_t)rl32((uint32_t)e.owner, w); ost = rl32((uint32_t)e.dstate, w);
        onsh = rl32((uint32_t)e.nsh, w); osh = 0; oh = (int32_t)i; od = false;
      }
      return (int32_t)i;
    }
    const uint64_t rv = ln < nrep ? rep_ent(ln)->addr : 0;
    const uint64_t rh = __ballot(ln < nrep && rv == a);
    if (rh) return -(int32_t)__builtin_ctzll(rh) - 1;
    return NO_ENT;
  }
  // replaceDirectoryEntry (directory_cache.cc:163-213): the slot gets a fresh
  // entry, the old one moves to the replaced list
  __device__ __forceinline__ int32_t dreplace(uint64_t replaced, uint64_t a, uint64_t& t)
  {
    eclose();                                     // the moves below work on HBM
    const uint32_t base = dset(replaced) * P.dassoc;
    DEnt* d = dirb;
    const uint64_t v = ln < P.dassoc ? d[base + ln].addr : 0;
    const uint64_t m = __ballot(ln < P.dassoc && v == replaced);
    if (!m) { fail(); return NO_ENT; }
    const int32_t slot = (int32_t)(base + __builtin_ctzll(m));
    const uint32_t r = nrep;
    if (r >= P.R) { fail(GG_DERR_CAP); return NO_ENT; }
    nrep = r + 1;
    *ent(-(int32_t)r - 1) = d[slot];
    uint64_t* so = shw(slot); uint64_t* sr = shw(-(int32_t)r - 1);
    for (uint32_t w = 0; w < wd; ++w) { sr[w] = so[w]; so[w] = 0; }
    d[slot] = DEnt{a, -1, DS_UNCACHED, 0};
    if constexpr (MO) {                           // the old entry keeps its Random, the new one is fresh
      S.rrng[(size_t)lt * P.R + r] = S.drng[(size_t)lt * P.E + slot];
      S.drng[(size_t)lt * P.E + slot] = 0;
    }
    t += P.lat_dir;
    stat(GG_CT_DIR_ACCESSES, 1);
    stat(GG_CT_DIR_EVICTIONS, 1);
    if (ent(-(int32_t)r - 1)->dstate != DS_UNCACHED) stat(GG_CT_DIR_BACK_INVALIDATIONS, 1);
    return slot;
  }
  // invalidateDirectoryEntry (directory_cache.cc:215-231): erase from the replaced list
  __device__ __forceinline__ void dinvalidate(uint64_t a)
  {
    eclose();                                     // the moves below work on HBM
    const uint32_t nr = nrep;
    const uint64_t rv = ln < nr ? rep_ent(ln)->addr : 0;
    const uint64_t rh = __ballot(ln < nr && rv == a);
    if (!rh) { fail(); return; }
    for (uint32_t k = (uint32_t)__builtin_ctzll(rh); k + 1 < nr; ++k) {
      *ent(-(int32_t)k - 1) = *ent(-(int32_t)k - 2);
      uint64_t* dst = shw(-(int32_t)k - 1); const uint64_t* src = shw(-(int32_t)k - 2);
      for (uint32_t w = 0; w < wd; ++w) dst[w] = src[w];
      if constexpr (MO) S.rrng[(size_t)lt * P.R + k] = S.rrng[(size_t)lt * P.R + k + 1];
    }
    nrep = nr - 1;
  }
  // getSharersList (ascending, full_map.cc:48-66): one message per sharer,
  // lane k writes the messages of sharer word k
  __device__ __forceinline__ void send_sharers(int32_t h, uint32_t type, uint32_t requester, uint64_t a, uint64_t t,
                                               uint32_t single_rx = 0)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; send_sharers_(h, type, requester, a, t, single_rx); if (tr_on) tra[1] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void send_sharers_(int32_t h, uint32_t type, uint32_t requester, uint64_t a, uint64_t t,
                                                uint32_t single_rx)
  {
    eopen(h);
    uint64_t bits = ln < wd ? osh : 0;
    const uint32_t c = (uint32_t)__builtin_popcountll(bits);
    const uint32_t pre = wave_excl_scan(c, ln);
    const uint32_t tot = wave_sum(c);
    if (!tot) return;
    const uint32_t base = alloc(tot);
    if (base == ~0u) return;
    uint32_t k = pre;
    while (bits) {
      const uint32_t b = (uint32_t)__builtin_ctzll(bits); bits &= bits - 1;
      put(base + k, ln * 64 + b, type, requester, a, t, seq + k, single_rx);
      ++k;
    }
    seq += tot;
    count_sent(type, tot);
  }

  // ---- per-address request FIFO (HashMapList<IntPtr, ShmemReq*>) -----------
  // Every access branches on rq_lds with each side's pointer typed by its
  // address space: a pointer merged from the two would compile to flat
  // accesses, and a flat access waits for every store the step has in flight
  __device__ __forceinline__ GG_LDS CReq* lrq() const { return (GG_LDS CReq*)sl.rq; }
  __device__ __forceinline__ uint64_t rq_addr(uint32_t i) const { return rq_lds ? lrq()[i].addr : rqg[i].addr; }
  __device__ __forceinline__ CReq rq_get(uint32_t i) const
  {
    if (rq_lds) { const GG_LDS CReq* x = lrq() + i; return CReq{x->addr, x->time, x->type, x->requester}; }
    const GG_GLB CReq* x = rqg + i;
    return CReq{x->addr, x->time, x->type, x->requester};
  }
  __device__ __forceinline__ void rq_put(uint32_t i, const CReq& v)
  {
    if (rq_lds) { GG_LDS CReq* x = lrq() + i; x->addr = v.addr; x->time = v.time; x->type = v.type; x->requester = v.requester; }
    else { GG_GLB CReq* x = rqg + i; x->addr = v.addr; x->time = v.time; x->type = v.type; x->requester = v.requester; }
  }
  // MOSI: the FIFO's other request fields (HBM)
  __device__ __forceinline__ CReqX rqx_get(uint32_t i) const
  {
    const GG_GLB CReqX* x = rqx + i;
    return CReqX{x->arrival, x->start, x->ds0, x->upg, x->sharer, 0};
  }
  __device__ __forceinline__ void rqx_put(uint32_t i, const CReqX& v)
  {
    GG_GLB CReqX* x = rqx + i;
    x->arrival = v.arrival; x->start = v.start; x->ds0 = v.ds0; x->upg = v.upg; x->sharer = v.sharer;
  }
  __device__ __forceinline__ uint32_t qcount(uint64_t a) const
  {
    uint32_t c = 0;                                  // a ballot per 64 entries (no cross-lane reduction)
    for (uint32_t b = 0; b < nrq; b += 64) c += (uint32_t)__builtin_popcountll(__ballot(b + ln < nrq && rq_addr(b + ln) == a));
    return c;
  }
  __device__ __forceinline__ int32_t qfront(uint64_t a) const
  {
    for (uint32_t b = 0; b < nrq; b += 64) {
      const uint32_t i = b + ln;
      const uint64_t m = __ballot(i < nrq && rq_addr(i) == a);
      if (m) return (int32_t)(b + __builtin_ctzll(m));
    }
    return -1;
  }
  __device__ __forceinline__ void qpush(uint64_t a, uint64_t t, uint32_t type, uint32_t req)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; qpush_(a, t, type, req); if (tr_on) tra[4] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void qpush_(uint64_t a, uint64_t t, uint32_t type, uint32_t req)
  {
    if (nrq >= (rq_lds ? SL::kRq : P.QC)) { fail(GG_DERR_CAP); return; }
    rq_put(nrq, CReq{a, t, type, req});
    if constexpr (MO) rqx_put(nrq, CReqX{t, t, DS_UNCACHED, 0, -1, 0});   // ShmemReq(msg, time) (…mosi/shmem_req.cc:8-22)
    if (rq_lds) wave_sync();
    ++nrq;
  }
  __device__ __forceinline__ void qpop(uint64_t a)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; qpop_(a); if (tr_on) tra[4] += __builtin_amdgcn_s_memtime() - c0; }
  __device__ __forceinline__ void qpop_(uint64_t a)
  {
    const int32_t f = qfront(a);
    if (f < 0) return;
    if (rq_lds) {                                   // shift down in LDS, lane-parallel
      for (uint32_t b = (uint32_t)f + 1; b < nrq; b += 64) {
        const uint32_t i = b + ln;
        CReq v{};
        if (i < nrq) v = rq_get(i);
        wave_sync();
        if (i < nrq) rq_put(i - 1, v);
        wave_sync();
      }
    } else {
      for (uint32_t k = (uint32_t)f; k + 1 < nrq; ++k) rq_put(k, rq_get(k + 1));
    }
    if constexpr (MO) {                             // the MOSI fields move with their entries
      for (uint32_t b = (uint32_t)f + 1; b < nrq; b += 64) {
        const uint32_t i = b + ln;
        CReqX v{};
        if (i < nrq) v = rqx_get(i);
        if (i < nrq) rqx_put(i - 1, v);               // (the loads of the 64 complete before any store)
      }
    }
    --nrq;
  }
  __device__ __forceinline__ static void front_time(CReq& r, uint64_t& t)   // ShmemReq::updateTime + updateCurrTime
  {
    if (r.time < t) r.time = t;
    if (t < r.time) t = r.time;
  }
  __device__ __forceinline__ void front_update(int32_t f, uint64_t& t, uint32_t& type, uint32_t& requester)
  {
    CReq r = rq_get(f);
    front_time(r, t);
    if (rq_lds) wave_sync();
    if (rq_lds) lrq()[f].time = r.time; else rqg[f].time = r.time;
    if (rq_lds) wave_sync();
    type = r.type; requester = r.requester;
  }

  // ---- DramCntlr / DramPerfModel --------------------------------------------
  __device__ __forceinline__ uint64_t dram_ps(uint64_t t)
  { const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0; const uint64_t r_ = dram_ps_(t); if (tr_on) tra[2] += __builtin_amdgcn_s_memtime() - c0; return r_; }
  __device__ __forceinline__ uint64_t dram_ps_(uint64_t t)
  {
    const uint64_t pkt_ns = time_to_cycles(t, 1.0);                  // ceil(t / 1000.0)
    uint64_t qd = 0;
    if (P.dram_qm) {
      // each side's queue pointers derived where they are used (LDS / HBM):
      // a pointer merged from the two would make every queue access flat
      if (F || (dq_lds && P.dram_qtype == GG_QM_HISTORY_TREE)) {
        // a history tree: the image into registers (RegQueue), one request,
        // back to the image — ~3x fewer cycles than the lane-parallel LDS form
        HQueue* lq = reinterpret_cast<HQueue*>(sl.dimg);
        HNode* lnd = reinterpret_cast<HNode*>(sl.dimg + sizeof(HQueue));
        RegQueue rq;
        rq.load_h0(lq, lnd, P.max_list, P.dram_proc, P.analytical != 0, ln);
        qd = rq.request(pkt_ns, P.dram_proc, S.err);
        wave_sync();
        rq.store(lq, lnd);
        wave_sync();
      } else if constexpr (!F) {
        if (dq_lds) {
          HTree tr{reinterpret_cast<HQueue*>(sl.dimg), reinterpret_cast<HNode*>(sl.dimg + sizeof(HQueue)), P.dram_proc,
                   P.analytical != 0};
          qd = tr.delay_w(pkt_ns, P.dram_proc, S.err, ln);
        } else {
          HTree tr{S.dq + lt, S.dnd + (size_t)lt * P.max_list, P.dram_proc, P.analytical != 0};
          qd = tr.delay(pkt_ns, P.dram_proc, S.err);
        }
      }
      stat(GG_CT_DRAM_QUEUE_REQUESTS, 1);
    }
    const uint64_t lat = qd + P.dram_proc + P.dram_cost;
    stat(GG_CT_DRAM_ACCESSES, 1);
    stat(GG_CT_DRAM_LATENCY_NS, lat);
    stat(GG_CT_DRAM_QUEUE_DELAY_NS, qd);
    return lat_to_ps(lat, 1.0);
  }

  // ---- DramDirectoryCntlr: the call chains as a work loop -------------------
  __device__ __forceinline__ void directory_run(Work w, uint64_t& t)
  {
    Work* stack = sl.wstack;                 // LDS: every lane writes / reads the same entry
    int sp = 0;
    for (;;) {
      if (failed) return;
      switch (w.kind) {
      case W_PROC: {                     // processEx/ShReqFromL2Cache (:238-380): entry lookup
        int32_t h = dget(w.addr, t);
        if (h == NO_ENT) {               // processDirectoryEntryAllocationReq (:126-170)
          const uint64_t msg_time = t;
          if (dget(w.addr, t) != NO_ENT) fail();   // the assert in getReplacementCandidates (directory_cache.cc:161)
          const uint32_t base = dset(w.addr) * P.dassoc;
          const DEnt* d = dirb;
          eflush();                                 // the scan reads the ways' sharer counts from HBM
          // candidate (:138-149): fewest sharers among ways with no queued request, first wins
          uint32_t key = ~0u;
          if (ln < P.dassoc) {
            const DEnt e = d[base + ln];
            uint32_t qc = 0;
            for (uint32_t i = 0; i < nrq; ++i) qc += (rq_addr(i) == e.addr);
            if (qc == 0) key = ((uint32_t)e.nsh << 8) | ln;
          }
          key = wave_min(key);
          if (key == ~0u) { fail(); return; }
          const uint64_t replaced = d[base + (key & 0xFFu)].addr;
          h = dreplace(replaced, w.addr, t);
          if (h == NO_ENT) return;
          qpush(replaced, msg_time, M_NULLIFY_REQ, w.requester);
          if (qcount(replaced) != 1) fail();
          if (sp >= WSTACK) { fail(GG_DERR_CAP); return; }
          Work c = w; c.kind = W_CONT; c.h = h;
          stack[sp++] = c;
          w = Work{replaced, W_NULLIFY, 0, w.requester, 0, 0};
          continue;
        }
        w.kind = W_CONT; w.h = h;
        continue;
      }
      case W_CONT: {                     // the directory-state switch
        const uint32_t ds = e_state(w.h);
        if (w.type == M_EX_REQ) {
          if (ds == DS_MODIFIED) {
            if (w.cached) fail();
            send((uint32_t)e_owner(w.h), M_FLUSH_REQ, w.requester, w.addr, t);
            w.kind = W_NONE;
          } else if (ds == DS_SHARED) {
            if (w.cached) fail();
            send_sharers(w.h, M_INV_REQ, w.requester, w.addr, t);
            w.kind = W_NONE;
          } else {
            add_sharer(w.h, w.requester);
            set_owner(w.h, (int32_t)w.requester);
            set_state(w.h, DS_MODIFIED);
            if (!w.cached) t += dram_ps(t);                         // retrieveDataAndSendToL2Cache (:382-408)
            send(w.requester, M_EX_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        } else {
          if (ds == DS_MODIFIED) {
            if (w.cached) fail();
            send((uint32_t)e_owner(w.h), M_WB_REQ, w.requester, w.addr, t);
            w.kind = W_NONE;
          } else {
            add_sharer(w.h, w.requester);
            set_state(w.h, DS_SHARED);
            if (!w.cached) t += dram_ps(t);
            send(w.requester, M_SH_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        }
        continue;
      }
      case W_NEXT: {                     // processNextReqFromL2Cache (:98-124)
        if (qcount(w.addr) < 1) { fail(); return; }
        qpop(w.addr);
        const int32_t f = qfront(w.addr);
        if (f < 0) { w.kind = W_NONE; continue; }
        uint32_t type, req;
        front_update(f, t, type, req);
        if (type != M_EX_REQ && type != M_SH_REQ) { fail(); return; }
        w = Work{w.addr, W_PROC, type, req, 0, 0};
        continue;
      }
      case W_NULLIFY: {                  // processNullifyReq (:172-236)
        const int32_t h = dget(w.addr, t);
        if (h == NO_ENT) { fail(); return; }
        const uint32_t ds = e_state(h);
        if (ds == DS_MODIFIED) {
          send((uint32_t)e_owner(h), M_FLUSH_REQ, w.requester, w.addr, t);
          w.kind = W_NONE;
        } else if (ds == DS_SHARED) {
          send_sharers(h, M_INV_REQ, w.requester, w.addr, t);
          w.kind = W_NONE;
        } else {
          dinvalidate(w.addr);
          w.kind = W_NEXT;
        }
        continue;
      }
      default:
        if (sp == 0) return;
        w = stack[--sp];
        continue;
      }
    }
  }

  // handleMsgFromL2Cache (:43-96) + processInv/Flush/WbRepFromL2Cache (:410-543)
  __device__ __forceinline__ void directory_msg(const HMsg& m)
  {
    const uint64_t c0 = tr_on ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t t = m.arrival_ps;           // __handleMsgFromNetwork: setCurrTime(packet.time)
    const uint64_t a = m.addr;
    Work w{a, W_NONE, 0, 0, 0, 0};
    if (m.type == M_EX_REQ || m.type == M_SH_REQ) {
      qpush(a, t, m.type, m.requester);
      if (qcount(a) == 1) w = Work{a, W_PROC, m.type, m.requester, 0, 0};
    } else {
      const int32_t h = dget(a, t);
      if (h == NO_ENT) { fail(); return; }
      const uint32_t ds = e_state(h);
      if (m.type == M_INV_REP) {
        if (ds != DS_SHARED) { fail(); return; }
        remove_sharer(h, m.src);
        const bool unc = e_nsh(h) == 0;
        if (unc) set_state(h, DS_UNCACHED);
        const int32_t f = qfront(a);
        if (f >= 0) {
          uint32_t type, req;
          front_update(f, t, type, req);
          if (type == M_EX_REQ) { if (unc) w = Work{a, W_PROC, M_EX_REQ, req, 0, 0}; }
          else if (type == M_SH_REQ) w = Work{a, W_PROC, M_SH_REQ, req, 0, 0};
          else { if (unc) w = Work{a, W_NULLIFY, 0, req, 0, 0}; }
        }
      } else if (m.type == M_FLUSH_REP) {
        if (ds != DS_MODIFIED) { fail(); return; }
        remove_sharer(h, m.src);
        set_owner(h, -1);
        set_state(h, DS_UNCACHED);
        const int32_t f = qfront(a);
        if (f < 0) { (void)dram_ps(t); return; }                    // putDataToDram: queue model, no latency
        uint32_t type, req;
        front_update(f, t, type, req);
        if (type == M_EX_REQ) w = Work{a, W_PROC, M_EX_REQ, req, 1, 0};
        else if (type == M_SH_REQ) { (void)dram_ps(t); w = Work{a, W_PROC, M_SH_REQ, req, 1, 0}; }
        else { (void)dram_ps(t); w = Work{a, W_NULLIFY, 0, req, 0, 0}; }
      } else if (m.type == M_WB_REP) {
        if (ds != DS_MODIFIED || !has(h, m.src)) { fail(); return; }
        set_owner(h, -1);
        set_state(h, DS_SHARED);
        const int32_t f = qfront(a);
        if (f < 0) { fail(); return; }
        uint32_t type, req;
        front_update(f, t, type, req);
        (void)dram_ps(t);
        if (type != M_SH_REQ) { fail(); return; }
        w = Work{a, W_PROC, M_SH_REQ, req, 1, 0};
      } else {
        fail();
        return;
      }
    }
    const uint64_t c1 = tr_on ? __builtin_amdgcn_s_memtime() : 0;
    if (tr_on) tra[6] += c1 - c0;
    if (w.kind != W_NONE) directory_run(w, t);
    if (tr_on) tra[7] += __builtin_amdgcn_s_memtime() - c1;
  }

  // ---- L1 / L2 controllers ---------------------------------------------------
  __device__ __forceinline__ void l1_invalidate(uint64_t a)                          // l1_cache_cntlr.cc:293-305
  {
    uint32_t s, l;
    L1.get(a, s, l);
    if (s != ST_I && !L1.set(a, ST_I, 0)) fail();
  }
  __device__ __forceinline__ void l1_access(uint64_t a, bool wr)                    // l1:182-205 (+ write-through, l2:66-70)
  {
    if (!L1.access(a, wr)) fail();
    if (wr && !L2.access(a, true)) fail();
  }
  __device__ __forceinline__ void insert_in_l1(uint64_t a, uint32_t cs)             // l2_cache_cntlr.cc:133-165
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L1.insert(a, cs, 0, ev, ea, es, el)) { fail(); return; }
    if (ev) {
      uint32_t s2, l2;
      L2.get(ea, s2, l2);
      if (l2 != 1) { fail(); return; }                               // cached_loc must be L1-D
      if (!L2.set(ea, s2, 0)) fail();                                // clearCachedLoc
    }
  }
  __device__ __forceinline__ void l2_insert(uint64_t a, uint32_t cs, uint64_t t)    // l2_cache_cntlr.cc:74-116
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L2.insert(a, cs, 1, ev, ea, es, el)) { fail(); return; }
    if (ev) {
      if (el) l1_invalidate(ea);
      if (es == ST_M) send(home(ea), M_FLUSH_REP, tile, ea, t);
      else if (es == ST_S) send(home(ea), M_INV_REP, tile, ea, t);
      else fail();
    }
  }
  __device__ __forceinline__ void finish(uint64_t start, uint64_t end, uint32_t level)
  {
    const uint64_t r = rec;
    const uint64_t lat = end - start;
    if (S.out) S.out[r] = (lat << 2) | level;
    stat(GG_CT_ACCESSES, 1);
    stat(GG_CT_LATENCY_PS, lat);
    if (level == GG_LVL_L1) stat(GG_CT_L1_HITS, 1); else if (level == GG_LVL_L2) stat(GG_CT_L2_HITS, 1); else stat(GG_CT_L2_MISSES, 1);
    clk = end;
    rec = r + 1;
  }
  // A run of L1 hits, one record per lane (records wbase + lane, window from
  // lane o).  Until the next miss nothing changes the L1 tags or states (a hit
  // only ages the LRU bits), so every lane looks its record up at once; the
  // issue times are a prefix sum (s = clk + gap, clk = s + lat_l1d on a hit);
  // the leading run of hits before the lax barrier is then retired in order:
  // the LRU touches (L1, and L2 for write-through stores) one by one, the
  // counters, statistics and access words in bulk.  Exactly app_access's hit
  // path applied record by record.  Returns the number of records retired.
  __device__ __forceinline__ uint32_t l1_hit_run(uint64_t wbase, uint32_t o, uint64_t wa, uint32_t wm, uint64_t line_mask,
                                                 uint64_t barrier)
  {
    const uint64_t a = wa & line_mask;
    const bool wr = (wm & GG_META_WRITE) != 0;
    const bool mine = ln >= o && wbase + ln < rec_end && wm != GG_META_BARRIER;
    bool hit = false, l2ok = true;
    uint32_t s1 = 0, w1 = 0, s2 = 0, w2 = 0;
    const bool rows = L1.ways <= 16 && L2.ways <= 16 && !P.touch_each;
    uint64_t r1a = 0, r1b = 0, r2a = 0, r2b = 0;                     // the record's set rows of meta bytes
    if (mine) {
      s1 = L1.set_of(a);
      const uint64_t tg = L1.tag_of(a);
      const uint64_t* tr = L1.tag + (size_t)s1 * L1.ways;
      int fw = -1;
#pragma unroll 8
      for (uint32_t w = 0; w < L1.ways; ++w) fw = tr[w] == tg ? (int)w : fw;   // independent loads, tags unique
      if (rows) load_row(L1.meta + (size_t)s1 * L1.ways, L1.ways, r1a, r1b);
      if (fw >= 0) {
        const uint32_t cs = (rows ? row_byte(r1a, r1b, (uint32_t)fw) : L1.meta[(size_t)s1 * L1.ways + fw]) & 3u;
        hit = wr ? cs == ST_M : cs != ST_I;
        w1 = (uint32_t)fw;
      }
      if (!SH && hit && wr) {                                        // the write-through L2 line (l2:66-70)
        s2 = L2.set_of(a);
        const uint64_t* t2 = L2.tag + (size_t)s2 * L2.ways;
        int f2 = -1;
#pragma unroll 8
        for (uint32_t w = 0; w < L2.ways; ++w) f2 = t2[w] == tg ? (int)w : f2;
        l2ok = f2 >= 0;                                              // absent: the general path fails as the reference asserts
        w2 = (uint32_t)f2;
        if (rows) load_row(L2.meta + (size_t)s2 * L2.ways, L2.ways, r2a, r2b);
      }
    }
    // end times: e = clk + gap_ps * (inclusive sum of gaps) + lat_l1d * (records so far)
    const uint32_t g = mine ? (wm & 0x7FFFFFFFu) >> 1 : 0;
    uint64_t e;
    if (!__ballot(g >= (1u << 25))) {
      e = (uint64_t)wave_incl_scan32(g) * P.gap_ps;
    } else {
      e = (uint64_t)g * P.gap_ps;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t v = shfl64(e, (int)ln - d);
        if ((int)ln >= d) e += v;
      }
    }
    e += clk + (uint64_t)(ln - o + 1) * P.lat_l1d;                   // this record's end time if all before it hit
    const bool ok = mine && hit && l2ok && (e - P.lat_l1d < barrier || (wm & GG_META_CONT));
    const uint64_t m = __ballot(ok) >> o;
    const uint32_t n = ~m ? (uint32_t)__builtin_ctzll(~m) : 64u - o;
    if (DG(S.prof) && ln == 0) { atomicAdd(&DG(S.prof)[37], (unsigned long long)__builtin_amdgcn_s_memtime()); atomicAdd(&DG(S.prof)[38], 1ull); }
    if (!n) return 0;
    const uint64_t run = (n == 64 ? ~0ull : ((1ull << n) - 1)) << o;
    const bool inrun = (run >> ln) & 1;
    const uint64_t wmask = __ballot(wr) & run;
    const uint32_t nw = (uint32_t)__builtin_popcountll(wmask);
    const bool lru1 = L1.pol == GG_POLICY_LRU, lru2 = !SH && L2.pol == GG_POLICY_LRU && nw;
    if ((lru1 || lru2) && rows) {
      // the run's LRU touches (lru:40-50) in closed form: ages are a
      // permutation of 0..ways-1 in every set (reset to the way index; touch
      // and insert permute them), so after the run a touched way's age is the
      // number of distinct ways of its set touched after its last touch, and an
      // untouched way i gets a_i + #{touched t: a_t > a_i}.  Lane = record:
      // tm = ways of my set touched in the run, af = those touched after me.
      uint32_t tm1 = 0, af1 = 0, tm2 = 0, af2 = 0;
      const bool w2l = inrun && wr;
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t l = o + k;
        if (lru1) {
          const uint32_t bit = 1u << rl32(w1, l);
          const bool same = s1 == rl32(s1, l);
          tm1 |= same ? bit : 0u;
          af1 |= same && l > ln ? bit : 0u;
        }
        if (lru2 && ((wmask >> l) & 1)) {
          const uint32_t bit = 1u << rl32(w2, l);
          const bool same = s2 == rl32(s2, l);
          tm2 |= same ? bit : 0u;
          af2 |= same && l > ln ? bit : 0u;
        }
      }
      PROF_AT(_q1);
      if (DG(S.prof) && ln == 0) atomicAdd(&DG(S.prof)[40], (unsigned long long)_q1);
      if (lru1 && inrun) lru_run_store(L1.meta + (size_t)s1 * L1.ways, L1.ways, r1a, r1b, w1, tm1, af1);
      if (lru2 && w2l) lru_run_store(L2.meta + (size_t)s2 * L2.ways, L2.ways, r2a, r2b, w2, tm2, af2);
      L1.cset = ~0u; L2.cset = ~0u;                                  // the one-row caches reload
      PROF_AT(_q2);
      if (DG(S.prof) && ln == 0) { atomicAdd(&DG(S.prof)[41], (unsigned long long)_q2); atomicAdd(&DG(S.prof)[42], 1ull); }
    } else if (lru1 || lru2) {                                       // > 16 ways: one touch at a time
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t l = o + k;
        uint64_t tv;
        uint32_t mv;
        if (lru1) { const uint32_t sk = rl32(s1, l); L1.ld(sk, tv, mv); L1.touch(sk, (int)rl32(w1, l), mv); }
        if (lru2 && ((wmask >> l) & 1)) { const uint32_t sk = rl32(s2, l); L2.ld(sk, tv, mv); L2.touch(sk, (int)rl32(w2, l), mv); }
      }
    }
    const uint32_t nr = n - nw;
    L1.cnt_add(GG_CC_TAG_READS, n);
    L1.cnt_add(GG_CC_ACCESSES, n);
    L1.cnt_add(GG_CC_READ_ACCESSES, nr);
    L1.cnt_add(GG_CC_WRITE_ACCESSES, nw);
    L1.cnt_add(GG_CC_DATA_READS, nr);
    L1.cnt_add(GG_CC_DATA_WRITES, nw);
    if constexpr (!SH) L2.cnt_add(GG_CC_DATA_WRITES, nw);
    if (S.out && ln >= o && ln < o + n) S.out[wbase + ln] = ((uint64_t)P.lat_l1d << 2) | GG_LVL_L1;
    stat(GG_CT_ACCESSES, n);
    stat(GG_CT_LATENCY_PS, (uint64_t)n * P.lat_l1d);
    stat(GG_CT_L1_HITS, n);
    clk = rl64(e, o + n - 1);
    rec += n;
    return n;
  }
  // Core::initiateMemoryAccess -> L1CacheCntlr::processMemOpFromCore, first attempt (l1:89-180)
  __device__ __forceinline__ void app_access(uint64_t a, bool wr, uint64_t s)
  {
    if constexpr (SH) { sh_app_access(a, wr, s); return; }
    uint64_t t = s;
    uint32_t cs, loc;
    L1.get(a, cs, loc);
    const bool hit = wr ? cs == ST_M : cs != ST_I;
    L1.miss_counters(a, wr, !hit);
    if (hit) { t += P.lat_l1d; l1_access(a, wr); finish(s, t, GG_LVL_L1); return; }
    t += P.lat_l1t;
    if constexpr (!MO) l1_invalidate(a);                             // (MOSI keeps the line, …mosi/l1:127-135)
    uint32_t c2, l2;                                                 // processShmemRequestFromL1Cache (l2:180-224)
    L2.get(a, c2, l2);
    const bool hit2 = wr ? c2 == ST_M : c2 != ST_I;
    L2.miss_counters(a, wr, !hit2);
    if (hit2) {
      if (!L2.access(a, false)) fail();
      insert_in_l1(a, c2);
      if (!L2.set(a, c2, 1)) fail();                                 // set(Forced)CachedLoc(L1-D)
      t += P.lat_l2d; t += P.lat_l1d;
      l1_access(a, wr);
      finish(s, t, GG_LVL_L2);
      return;
    }
    t += P.lat_l2t;
    if (out_addr != INV_ADDR) fail();                                // handleMsgFromL1Cache (l2:226-258)
    out_addr = a; out_time = t;
    const uint32_t h = home(a);
    if constexpr (MO) {                                              // …mosi/l2:266-285: the request as is
      send(h, wr ? M_EX_REQ : M_SH_REQ, tile, a, t);
    } else if (wr) {                                                 // processExReqFromL1Cache (l2:260-282)
      uint32_t x, xl;
      L2.get(a, x, xl);
      if (x == ST_S) { if (!L2.set(a, ST_I, 0)) fail(); send(h, M_INV_REP, tile, a, t); }
      else if (x != ST_I) fail();
      send(h, M_EX_REQ, tile, a, t);
    } else {
      send(h, M_SH_REQ, tile, a, t);
    }
    blocked = 1;
    pend_start = s;
  }
  // L2CacheCntlr::handleMsgFromDramDirectory (l2:294-502) + the core's second attempt
  __device__ __forceinline__ void l2_msg(const HMsg& m)
  {
    uint64_t t = m.arrival_ps;
    const uint64_t a = m.addr;
    if (m.type == M_EX_REP || m.type == M_SH_REP) {
      const uint32_t cs = m.type == M_EX_REP ? ST_M : ST_S;
      if (!blocked || out_addr != a) { fail(); return; }
      l2_insert(a, cs, t);
      insert_in_l1(a, cs);
      if (out_time > t) fail();
      t += P.lat_l2d;
      out_addr = INV_ADDR;
      const bool wr = (S.meta[rec] & GG_META_WRITE) != 0;     // access_num == 2 (l1:106-126)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      const bool hit = wr ? c1 == ST_M : c1 != ST_I;
      if (!hit) { fail(); return; }
      t += P.lat_l1d;
      l1_access(a, wr);
      blocked = 0;
      finish(pend_start, t, GG_LVL_DIR);
      return;
    }
    uint32_t c2, loc;
    L2.get(a, c2, loc);
    if (c2 == ST_I) { t += P.lat_l2t; return; }                      // line already gone: tags only, no reply
    if (m.type == M_INV_REQ) {                                       // l2:369-410
      if (c2 != ST_S) { fail(); return; }
      t += P.lat_l2t;
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_INV_REP, m.requester, a, t);
    } else if (m.type == M_FLUSH_REQ) {                              // l2:412-455
      if (c2 != ST_M) { fail(); return; }
      t += P.lat_l2d;
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_FLUSH_REP, m.requester, a, t);
    } else if (m.type == M_WB_REQ) {                                 // l2:457-502
      if (c2 != ST_M) { fail(); return; }
      t += P.lat_l2d;
      if (loc) {
        t += P.lat_l1t;
        uint32_t c1, l1;                                             // setCacheLineState (l1:278-291)
        L1.get(a, c1, l1);
        if (c1 == ST_I) fail();
        if (!L1.set(a, ST_S, 0)) fail();
      }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ST_S, loc)) fail();
      send(m.src, M_WB_REP, m.requester, a, t);
    } else {
      fail();
    }
  }

  // ==== MOSI (pr_l1_pr_l2_dram_directory_mosi) ================================
  // The MOSI directory and L2 controllers on the same directory cache, request
  // FIFO, DRAM, clock and network as the MSI ones above (Tile<..., MO = true>).
  __device__ __forceinline__ uint64_t* rng_ptr(int32_t h) const
  {
    h = __builtin_amdgcn_readfirstlane(h);
    return h >= 0 ? S.drng + (size_t)lt * P.E + h : S.rrng + (size_t)lt * P.R + (-h - 1);
  }
  // DirectoryEntryFullMap::getOneSharer (directory_entry_full_map.cc:67-74):
  // Random<int>::next(#sharers) over drand48_r (misc/random.h:25-31) —
  // X <- (0x5DEECE66D X + 0xB) mod 2^48, result X / 2^48 (exact in a double),
  // index (int)(result * n) — into the ascending sharers list (lane w holds
  // sharer word w: the index's word by a prefix count, its bit by clearing)
  __device__ __forceinline__ int32_t one_sharer(int32_t h)
  {
    eopen(h);
    uint64_t* rp = rng_ptr(h);
    uint64_t x = *rp ^ kRng0;
    x = (0x5DEECE66Dull * x + 0xBull) & 0xFFFFFFFFFFFFull;
    *rp = x ^ kRng0;
    const double r = (double)x * 0x1p-48;
    const uint32_t n = onsh;
    const uint32_t k = (uint32_t)(int)(r * (double)(int)n);
    if (k >= n) { fail(); return 0; }
    const uint64_t bits = ln < wd ? osh : 0ull;
    const uint32_t c = (uint32_t)__builtin_popcountll(bits);
    const uint32_t pre = wave_excl_scan(c, ln);
    const bool mine = k >= pre && k < pre + c;
    uint32_t sh = 0;
    if (mine) {
      uint64_t b = bits;
      for (uint32_t j = k - pre; j; --j) b &= b - 1;
      sh = ln * 64 + (uint32_t)__builtin_ctzll(b);
    }
    const uint64_t who = __ballot(mine);
    if (!who) { fail(); return 0; }
    return (int32_t)rl32(sh, (uint32_t)__builtin_ctzll(who));
  }
  // DataList (…mosi/dram_directory_cntlr.cc:1196-1241): the line data is not modeled
  __device__ __forceinline__ int32_t cdl_find(uint64_t a) const
  {
    if (!ncdl) return -1;
    const uint64_t v = ln < ncdl ? S.cdl[(size_t)lt * kCdl + ln] : 0ull;
    const uint64_t m = __ballot(ln < ncdl && v == a);
    return m ? (int32_t)__builtin_ctzll(m) : -1;
  }
  __device__ __forceinline__ void cdl_insert(uint64_t a)
  {
    if (cdl_find(a) >= 0) return;                                 // already there: the same data
    if (ncdl >= kCdl) { fail(GG_DERR_CAP); return; }
    S.cdl[(size_t)lt * kCdl + ncdl] = a;
    ++ncdl;
  }
  __device__ __forceinline__ void cdl_erase_at(int32_t i)
  {
    uint64_t* c = S.cdl + (size_t)lt * kCdl;
    const uint64_t last = c[ncdl - 1];
    c[i] = last;
    --ncdl;
  }
  // updateShmemReqEventCounters (:879-965) of the request at FIFO slot f, with
  // setInitialDState before it (first_call of process*Req)
  __device__ __forceinline__ void mo_event(int32_t h, int32_t f, uint32_t type, uint32_t requester)
  {
    const uint32_t ds = e_state(h), n = e_nsh(h);
    const bool shared = ds == DS_OWNED || ds == DS_SHARED;
    rqx[f].ds0 = ds;
    if (type == M_EX_REQ) {
      pstat(GG_PS_EXREQ);
      if (ds == DS_MODIFIED) pstat(GG_PS_EXREQ_MODIFIED);
      else if (shared) {
        pstat(GG_PS_EXREQ_SHARED);
        if (n == 1 && one_sharer(h) == (int32_t)requester) { rqx[f].upg = 1; pstat(GG_PS_EXREQ_UPGRADE); }
        else { pstat(GG_PS_INV_UNICAST); pstat(GG_PS_INV_SHARERS_UNICAST, n); }   // updateInvalidationEventCounters
      } else pstat(GG_PS_EXREQ_UNCACHED);
    } else if (type == M_SH_REQ) {
      pstat(GG_PS_SHREQ);
      pstat(ds == DS_MODIFIED ? GG_PS_SHREQ_MODIFIED : shared ? GG_PS_SHREQ_SHARED : GG_PS_SHREQ_UNCACHED);
    } else {
      pstat(GG_PS_NULLIFY);
      if (ds == DS_MODIFIED) pstat(GG_PS_NULLIFY_MODIFIED);
      else if (shared) { pstat(GG_PS_NULLIFY_SHARED); pstat(GG_PS_INV_UNICAST); pstat(GG_PS_INV_SHARERS_UNICAST, n); }
      else pstat(GG_PS_NULLIFY_UNCACHED);
    }
  }
  // the completed front of a FIFO: updateProcessingFinishTime + updateShmemReqLatencyCounters (:982-1014)
  __device__ __forceinline__ void mo_retire(int32_t f, uint64_t t)
  {
    const CReq r = rq_get(f);
    const CReqX x = rqx_get(f);
    const uint64_t fin = r.time < t ? t : r.time;
    const uint64_t ser = x.start - x.arrival, proc = fin - x.start;
    const bool inv0 = x.ds0 == DS_OWNED || x.ds0 == DS_SHARED;
    if (r.type == M_EX_REQ) {
      pstat(GG_PS_EXREQ_SERIALIZATION_PS, ser); pstat(GG_PS_EXREQ_PROCESSING_PS, proc);
      if (inv0 && !x.upg) pstat(GG_PS_INV_PROCESSING_UNICAST_PS, proc);
    } else if (r.type == M_SH_REQ) {
      pstat(GG_PS_SHREQ_SERIALIZATION_PS, ser); pstat(GG_PS_SHREQ_PROCESSING_PS, proc);
    } else {
      pstat(GG_PS_NULLIFY_SERIALIZATION_PS, ser); pstat(GG_PS_NULLIFY_PROCESSING_PS, proc);
      if (inv0) pstat(GG_PS_INV_PROCESSING_UNICAST_PS, proc);
    }
  }
  // retrieveDataAndSendToL2Cache (:563-595): the cached data, else DRAM
  __device__ __forceinline__ void mo_retrieve(uint32_t type, uint32_t rx, uint64_t a, uint64_t& t)
  {
    const int32_t ci = cdl_find(a);
    if (ci >= 0) { send(rx, type, rx, a, t); cdl_erase_at(ci); }
    else { t += dram_ps(t); send(rx, type, rx, a, t); }
  }
  // restartShmemReq (:797-833): the work item it continues with (W_NONE if none)
  __device__ __forceinline__ Work mo_restart(uint32_t sender, int32_t f, int32_t h, uint64_t a, uint64_t& t)
  {
    uint32_t type, req;
    front_update(f, t, type, req);                                  // updateProcessingFinishTime + updateCurrTime(getTime())
    const uint32_t ds = e_state(h);
    if (type == M_EX_REQ) return ds == DS_UNCACHED ? Work{a, W_CONT, M_EX_REQ, req, 0, h} : Work{a, W_NONE, 0, 0, 0, NO_ENT};
    if (type == M_SH_REQ) {
      const int32_t sh = rqx[f].sharer;
      if (sh < 0) { fail(); return Work{a, W_NONE, 0, 0, 0, NO_ENT}; }
      if ((int32_t)sender != sh) return Work{a, W_NONE, 0, 0, 0, NO_ENT};
      rqx[f].sharer = -1;
      return Work{a, W_CONT, M_SH_REQ, req, 0, h};
    }
    return ds == DS_UNCACHED ? Work{a, W_NULLIFY, 0, req, 0, h} : Work{a, W_NONE, 0, 0, 0, NO_ENT};
  }
  // the MOSI call chains as a work loop (Work::cached = first_call, Work::h =
  // the entry when the reference passes one, else NO_ENT)
  __device__ __forceinline__ void directory_run_mo(Work w, uint64_t& t)
  {
    Work* stack = sl.wstack;
    int sp = 0;
    for (;;) {
      if (failed) return;
      switch (w.kind) {
      case W_PROC: {                     // processEx/ShReqFromL2Cache (…mosi :299-533): no entry given
        int32_t h = dget(w.addr, t);
        if (h == NO_ENT) {               // processDirectoryEntryAllocationReq (:165-209)
          const uint64_t msg_time = t;
          if (dget(w.addr, t) != NO_ENT) fail();   // getReplacementCandidates' assert (directory_cache.cc:161)
          const uint32_t base = dset(w.addr) * P.dassoc;
          const DEnt* d = dirb;
          eflush();
          uint32_t key = ~0u;
          if (ln < P.dassoc) {
            const DEnt e = d[base + ln];
            uint32_t qc = 0;
            for (uint32_t i = 0; i < nrq; ++i) qc += (rq_addr(i) == e.addr);
            if (qc == 0) key = ((uint32_t)e.nsh << 8) | ln;
          }
          key = wave_min(key);
          if (key == ~0u) { fail(); return; }
          const uint64_t replaced = d[base + (key & 0xFFu)].addr;
          h = dreplace(replaced, w.addr, t);
          if (h == NO_ENT) return;
          qpush(replaced, msg_time, M_NULLIFY_REQ, w.requester);
          if (qcount(replaced) != 1) fail();
          if (sp >= WSTACK) { fail(GG_DERR_CAP); return; }
          Work c = w; c.kind = W_CONT; c.h = h;
          stack[sp++] = c;
          w = Work{replaced, W_NULLIFY, 0, w.requester, 1, NO_ENT};
          continue;
        }
        w.kind = W_CONT; w.h = h;
        continue;
      }
      case W_CONT: {                     // the directory-state switch
        const int32_t f = qfront(w.addr);
        if (f < 0) { fail(); return; }
        if (w.cached) mo_event(w.h, f, w.type, w.requester);
        const uint32_t ds = e_state(w.h), n = e_nsh(w.h);
        w.kind = W_NONE;
        if (w.type == M_EX_REQ) {
          if (ds == DS_MODIFIED) {
            send((uint32_t)e_owner(w.h), M_FLUSH_REQ, w.requester, w.addr, t);
          } else if (ds == DS_OWNED) {
            const int32_t o = e_owner(w.h);
            if (o == (int32_t)w.requester && n == 1) {
              set_state(w.h, DS_MODIFIED);
              send(w.requester, M_UPGRADE_REP, w.requester, w.addr, t);
              w.kind = W_NEXT;
            } else {
              send_sharers(w.h, M_IFC_REQ, w.requester, w.addr, t, (uint32_t)o);   // FLUSH to the owner, INV to the rest
            }
          } else if (ds == DS_SHARED) {
            if (n == 0) fail();
            if (n == 1 && has(w.h, w.requester)) {
              set_owner(w.h, (int32_t)w.requester);
              set_state(w.h, DS_MODIFIED);
              send(w.requester, M_UPGRADE_REP, w.requester, w.addr, t);
              w.kind = W_NEXT;
            } else {
              const int32_t one = one_sharer(w.h);
              send_sharers(w.h, M_IFC_REQ, w.requester, w.addr, t, (uint32_t)one);
            }
          } else {
            if (n != 0) fail();
            add_sharer(w.h, w.requester);
            set_owner(w.h, (int32_t)w.requester);
            set_state(w.h, DS_MODIFIED);
            mo_retrieve(M_EX_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        } else {
          if (ds == DS_MODIFIED) {
            const int32_t o = e_owner(w.h);
            send((uint32_t)o, M_WB_REQ, w.requester, w.addr, t);
            rqx[f].sharer = o;
          } else if (ds == DS_OWNED || ds == DS_SHARED) {
            if (n == 0) fail();
            const int32_t sh = one_sharer(w.h);            // the sharer can be the owner
            add_sharer(w.h, w.requester);
            if (cdl_find(w.addr) < 0) {
              remove_sharer(w.h, w.requester);             // not complete yet: the data comes from the sharer
              send((uint32_t)sh, M_WB_REQ, w.requester, w.addr, t);
              rqx[f].sharer = sh;
            } else {
              mo_retrieve(M_SH_REP, w.requester, w.addr, t);
              w.kind = W_NEXT;
            }
          } else {
            add_sharer(w.h, w.requester);
            set_state(w.h, DS_SHARED);
            mo_retrieve(M_SH_REP, w.requester, w.addr, t);
            w.kind = W_NEXT;
          }
        }
        w.h = NO_ENT;
        continue;
      }
      case W_NEXT: {                     // processNextReqFromL2Cache (…mosi :117-163)
        if (qcount(w.addr) < 1) { fail(); return; }
        mo_retire(qfront(w.addr), t);
        qpop(w.addr);
        if (cdl_find(w.addr) >= 0) fail();           // assert(_cached_data_list.lookup(address) == NULL)
        const int32_t f = qfront(w.addr);
        if (f < 0) { w.kind = W_NONE; continue; }
        // updateProcessingStartTime + updateCurrTime(getTime())
        CReq r = rq_get(f);
        if (rqx[f].start < t) {
          rqx[f].start = t; r.time = t;
          if (rq_lds) wave_sync();
          if (rq_lds) lrq()[f].time = t; else rqg[f].time = t;
          if (rq_lds) wave_sync();
        }
        if (t < r.time) t = r.time;
        if (r.type != M_EX_REQ && r.type != M_SH_REQ) { fail(); return; }
        w = Work{w.addr, W_PROC, r.type, r.requester, 1, NO_ENT};
        continue;
      }
      case W_NULLIFY: {                  // processNullifyReq (…mosi :211-297)
        const int32_t h = w.h != NO_ENT ? w.h : dget(w.addr, t);
        if (h == NO_ENT) { fail(); return; }
        if (w.cached) {
          const int32_t f = qfront(w.addr);
          if (f < 0) { fail(); return; }
          mo_event(h, f, M_NULLIFY_REQ, w.requester);
        }
        const uint32_t ds = e_state(h);
        w.h = NO_ENT;
        if (ds == DS_MODIFIED) {
          send((uint32_t)e_owner(h), M_FLUSH_REQ, w.requester, w.addr, t);
          w.kind = W_NONE;
        } else if (ds == DS_OWNED) {
          const int32_t o = e_owner(h);
          if (o < 0) fail();
          send_sharers(h, M_IFC_REQ, w.requester, w.addr, t, (uint32_t)o);
          w.kind = W_NONE;
        } else if (ds == DS_SHARED) {
          if (e_owner(h) >= 0) fail();
          send_sharers(h, M_INV_REQ, w.requester, w.addr, t);
          w.kind = W_NONE;
        } else {
          const int32_t ci = cdl_find(w.addr);
          if (ci >= 0) { (void)dram_ps(t); cdl_erase_at(ci); }      // sendDataToDram
          dinvalidate(w.addr);
          w.kind = W_NEXT;
        }
        continue;
      }
      default:
        if (sp == 0) return;
        w = stack[--sp];
        continue;
      }
    }
  }
  // handleMsgFromL2Cache (…mosi :49-115) + processInv/Flush/WbRepFromL2Cache (:597-795)
  __device__ __forceinline__ void directory_msg_mo(const HMsg& m)
  {
    uint64_t t = m.arrival_ps;
    const uint64_t a = m.addr;
    const uint32_t src = m.src;
    Work w{a, W_NONE, 0, 0, 0, NO_ENT};
    if (m.type == M_EX_REQ || m.type == M_SH_REQ) {
      qpush(a, t, m.type, m.requester);
      if (qcount(a) == 1) {
        if (cdl_find(a) >= 0) fail();
        w = Work{a, W_PROC, m.type, m.requester, 1, NO_ENT};
      }
    } else {
      const int32_t h = dget(a, t);
      if (h == NO_ENT) { fail(); return; }
      const uint32_t ds = e_state(h);
      if (m.type == M_INV_REP) {
        if (ds == DS_OWNED) {
          if ((int32_t)src == e_owner(h) || e_nsh(h) == 0) fail();
          remove_sharer(h, src);
          if (e_nsh(h) == 0) fail();
        } else if (ds == DS_SHARED) {
          if (e_owner(h) >= 0 || e_nsh(h) == 0) fail();
          remove_sharer(h, src);
          if (e_nsh(h) == 0) set_state(h, DS_UNCACHED);
        } else { fail(); return; }
        const int32_t f = qfront(a);
        if (f >= 0) w = mo_restart(src, f, h, a, t);
      } else if (m.type == M_FLUSH_REP) {
        if (ds == DS_MODIFIED) {
          if ((int32_t)src != e_owner(h)) fail();
          remove_sharer(h, src);
          set_owner(h, -1);
          set_state(h, DS_UNCACHED);
        } else if (ds == DS_OWNED) {
          const int32_t o = e_owner(h);
          if (o < 0 || e_nsh(h) == 0) fail();
          remove_sharer(h, src);
          if ((int32_t)src == o) { set_owner(h, -1); set_state(h, e_nsh(h) > 0 ? DS_SHARED : DS_UNCACHED); }
        } else if (ds == DS_SHARED) {
          if (e_owner(h) >= 0 || e_nsh(h) == 0) fail();
          remove_sharer(h, src);
          if (e_nsh(h) == 0) set_state(h, DS_UNCACHED);
        } else { fail(); return; }
        const int32_t f = qfront(a);
        if (f >= 0) {
          cdl_insert(a);
          const uint32_t ds1 = e_state(h);
          if (rq_get(f).type == M_SH_REQ && (ds == DS_MODIFIED || ds == DS_OWNED) && (ds1 == DS_SHARED || ds1 == DS_UNCACHED))
            (void)dram_ps(t);                                        // sendDataToDram
          w = mo_restart(src, f, h, a, t);
        } else {
          (void)dram_ps(t);                                          // just an eviction: to DRAM
        }
      } else if (m.type == M_WB_REP) {
        if (ds == DS_MODIFIED) {
          if ((int32_t)src != e_owner(h) || qcount(a) == 0) fail();
          set_state(h, DS_OWNED);
        } else if (ds == DS_OWNED) {
          if (!has(h, src)) fail();
        } else if (ds == DS_SHARED) {
          if (e_owner(h) >= 0 || !has(h, src)) fail();
        } else { fail(); return; }
        const int32_t f = qfront(a);
        if (f < 0) { fail(); return; }                                 // "WB_REP, NO requester"
        cdl_insert(a);
        w = mo_restart(src, f, h, a, t);
      } else {
        fail();
        return;
      }
    }
    if (w.kind != W_NONE) directory_run_mo(w, t);
  }
  // L2CacheCntlr::insertCacheLine (…mosi/l2_cache_cntlr.cc:95-149) + updateEvictionCounters (:605-636)
  __device__ __forceinline__ void l2_insert_mo(uint64_t a, uint32_t cs, uint64_t t)
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L2.insert(a, cs, 1, ev, ea, es, el)) { fail(); return; }
    if (!ev) return;
    const bool dirty = es == ST_M || es == ST_O;
    if (!dirty && es != ST_S) { fail(); return; }
    pstat(GG_PS_L2_EVICTIONS);
    pstat(cs == ST_M ? (dirty ? GG_PS_L2_DIRTY_EVICTIONS_EXREQ : GG_PS_L2_CLEAN_EVICTIONS_EXREQ)
                     : (dirty ? GG_PS_L2_DIRTY_EVICTIONS_SHREQ : GG_PS_L2_CLEAN_EVICTIONS_SHREQ));
    if (el) l1_invalidate(ea);
    send(home(ea), dirty ? M_FLUSH_REP : M_INV_REP, tile, ea, t);
  }
  // L2CacheCntlr::handleMsgFromDramDirectory (…mosi :287-594) + the core's second attempt
  __device__ __forceinline__ void l2_msg_mo(const HMsg& m)
  {
    uint64_t t = m.arrival_ps;
    const uint64_t a = m.addr;
    uint32_t type = m.type;
    if (type == M_IFC_REQ) type = m.single_rx == tile ? M_FLUSH_REQ : M_INV_REQ;   // (:581-594)
    if (type == M_EX_REP || type == M_SH_REP || type == M_UPGRADE_REP) {
      if (!blocked || out_addr != a) { fail(); return; }
      if (type != M_UPGRADE_REP) {                                   // insertCacheLineInHierarchy (:210-224)
        const uint32_t cs = type == M_EX_REP ? ST_M : ST_S;
        l2_insert_mo(a, cs, t);
        insert_in_l1(a, cs);
      } else {                                                       // processUpgradeRepFromDramDirectory (:370-412)
        uint32_t c2, loc;
        L2.get(a, c2, loc);
        if (c2 != ST_S && c2 != ST_O) fail();
        if (!loc) {
          if (!L2.access(a, false)) fail();                          // readCacheLine
          insert_in_l1(a, ST_M);
          loc = 1;
        } else {
          uint32_t c1, l1;                                           // setCacheLineState (…mosi/l1:260-273)
          L1.get(a, c1, l1);
          if (c1 == ST_I) fail();
          if (!L1.set(a, ST_M, 0)) fail();
        }
        if (!L2.set(a, ST_M, loc)) fail();
      }
      if (out_time > t) fail();
      t += P.lat_l2d;
      out_addr = INV_ADDR;
      const bool wr = (S.meta[rec] & GG_META_WRITE) != 0;          // access_num == 2 (…mosi/l1:105-126)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      const bool hit = wr ? c1 == ST_M : c1 != ST_I;
      if (!hit) { fail(); return; }
      t += P.lat_l1d;
      l1_access(a, wr);
      blocked = 0;
      finish(pend_start, t, GG_LVL_DIR);
      return;
    }
    uint32_t c2, loc;
    L2.get(a, c2, loc);
    if (c2 == ST_I) { t += P.lat_l2t; return; }                      // tags only; full map: no reply expected
    if (type == M_INV_REQ) {                                         // (:414-468)
      if (c2 != ST_S) { fail(); return; }
      t += P.lat_l2t;
      pstat(GG_PS_L2_INVALIDATIONS);
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_INV_REP, m.requester, a, t);
    } else if (type == M_FLUSH_REQ) {                                // (MODIFIED, OWNED, SHARED) -> INVALID (:470-527)
      t += P.lat_l2d;
      pstat(GG_PS_L2_INVALIDATIONS);
      if (loc) { t += P.lat_l1t; l1_invalidate(a); }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ST_I, 0)) fail();
      send(m.src, M_FLUSH_REP, m.requester, a, t);
    } else if (type == M_WB_REQ) {                                   // M -> O, O -> O, S -> S (:529-579)
      t += P.lat_l2d;
      const uint32_t ns = c2 == ST_M ? ST_O : c2;
      if (loc) {
        t += P.lat_l1t;
        uint32_t c1, l1;
        L1.get(a, c1, l1);
        if (c1 == ST_I) fail();
        if (!L1.set(a, ns, 0)) fail();
      }
      if (!L2.access(a, false)) fail();
      if (!L2.set(a, ns, loc)) fail();
      send(m.src, M_WB_REP, m.requester, a, t);
    } else {
      fail();
    }
  }

  // store-only write back of what the step changed: the counters were
  // loaded with the tile, and an idle tile (most of them in a step) leaves
  // its lines clean, so the launch's end writes back only the active tiles'
  // state (the agent-scope release costs by the dirty bytes)
  // ==== pr_l1_sh_l2_msi (Tile<..., PR = 2>) ====================================
  // The tile's L2 slice is its directory-entry array: slot set * a2 + way
  // holds one line (addr = its address, INV_ADDR while never used; dstate =
  // directory state | cache state << 8: DATA_INVALID, CLEAN or DIRTY; owner,
  // sharer count and words), set = L2CacheHashFn (the directory's XOR fold
  // over log2(sets)-bit fields, no slice bits); the replaced list is
  // L2CacheCntlr::_evicted_cache_line_map.  The slice's Cache operations count
  // in L2.cd.  The controller's call chains run as a work loop (sh_run), as
  // directory_run does for the private-L2 protocols.
  static constexpr uint32_t CS_DINV = 5, CS_CLEAN = 6, CS_DIRTY = 7;          // CacheState::Type (cache_state.h:11-22)
  enum { SW_NONE = 0, SW_PROC, SW_CONT, SW_NULL, SW_NEXT };
  struct SWork { uint64_t addr; uint32_t kind, type, first, data, req; int32_t h; };
  static_assert(sizeof(SWork) <= sizeof(Work), "SWork continuations live in the directory work stack");
  __device__ __forceinline__ uint32_t sh_cs(int32_t h) { return e_state(h) >> 8; }
  __device__ __forceinline__ uint32_t sh_ds(int32_t h) { return e_state(h) & 0xFFu; }
  __device__ __forceinline__ void sh_set_ds(int32_t h, uint32_t ds) { eopen(h); ost = (ost & 0xFF00u) | ds; od = true; }
  __device__ __forceinline__ void sh_set_cs(int32_t h, uint32_t cs) { eopen(h); ost = (ost & 0xFFu) | (cs << 8); od = true; }
  // CacheSet::find in the slice (lane = way): the line's slot or NO_ENT
  __device__ __forceinline__ int32_t sh_slot(uint64_t a)
  {
    const uint32_t base = dset(a) * P.dassoc;
    const DEnt* d = dirb;
    const uint64_t v = ln < P.dassoc ? d[base + ln].addr : INV_ADDR;
    const uint64_t m = __ballot(ln < P.dassoc && v == a);
    return m ? (int32_t)(base + (uint32_t)__builtin_ctzll(m)) : NO_ENT;
  }
  // _evicted_cache_line_map.find (lane = entry)
  __device__ __forceinline__ int32_t sh_evicted(uint64_t a)
  {
    const uint64_t rv = ln < nrep ? rep_ent(ln)->addr : INV_ADDR;
    const uint64_t rh = __ballot(ln < nrep && rv == a);
    return rh ? -(int32_t)__builtin_ctzll(rh) - 1 : NO_ENT;
  }
  // L2CacheCntlr::setCacheLineInfo (l2_cache_cntlr.cc:102-116): a line in the
  // slice is a tag write (its fields go back with the open entry)
  __device__ __forceinline__ void sh_setinfo(int32_t h) { if (h >= 0) L2.cnt(GG_CC_TAG_WRITES); }
  // allocateCacheLine (l2_cache_cntlr.cc:130-189): a DATA_INVALID line with a
  // fresh entry; the victim (L2CacheReplacementPolicy::getReplacementWay,
  // l2_cache_replacement_policy.cc:20-67: the first INVALID way, else the
  // fewest sharers among lines no request waits on, first wins) moves to the
  // evicted map.  Returns the new line's slot; ev_addr = the victim's line or INV_ADDR.
  __device__ __forceinline__ int32_t sh_allocate(uint64_t a, uint64_t& ev_addr)
  {
    eclose();                                     // the moves below work on HBM
    ev_addr = INV_ADDR;
    const uint32_t base = dset(a) * P.dassoc;
    DEnt* d = dirb;
    DEnt e{INV_ADDR, -1, 0, 0};
    if (ln < P.dassoc) e = d[base + ln];
    const uint64_t inv = __ballot(ln < P.dassoc && e.addr == INV_ADDR);
    uint32_t w;
    if (inv) {
      w = (uint32_t)__builtin_ctzll(inv);
    } else {
      uint32_t key = ~0u;
      if (ln < P.dassoc) {
        uint32_t qc = 0;
        for (uint32_t i = 0; i < nrq; ++i) qc += (rq_addr(i) == e.addr);
        if (qc == 0) key = ((uint32_t)e.nsh << 8) | ln;
      }
      key = wave_min(key);
      if (key == ~0u) { fail(); return NO_ENT; }  // "Could not find a replacement candidate"
      w = key & 0xFFu;
    }
    const int32_t slot = (int32_t)(base + w);
    const uint64_t va = rl64(e.addr, w);
    L2.cnt(GG_CC_TAG_READS);
    if (va != INV_ADDR) {
      const uint32_t r = nrep;
      if (r >= P.R) { fail(GG_DERR_CAP); return NO_ENT; }
      nrep = r + 1;
      *ent(-(int32_t)r - 1) = d[slot];
      uint64_t* so = shw(slot); uint64_t* sr = shw(-(int32_t)r - 1);
      if (ln < wd) sr[ln] = so[ln];
      const uint32_t vcs = rl32((uint32_t)e.dstate, w) >> 8;
      if (vcs != CS_CLEAN && vcs != CS_DIRTY) fail();
      L2.cnt(GG_CC_DATA_READS); L2.cnt(GG_CC_EVICTIONS);
      if (vcs == CS_DIRTY) L2.cnt(GG_CC_DIRTY_EVICTIONS);
      ev_addr = va;
    }
    d[slot] = DEnt{a, -1, (uint16_t)((CS_DINV << 8) | DS_UNCACHED), 0};
    if (ln < wd) shw(slot)[ln] = 0;
    L2.cnt(GG_CC_TAG_WRITES); L2.cnt(GG_CC_DATA_WRITES);
    return slot;
  }
  // processNextReqFromL1Cache (l2_cache_cntlr.cc:305-336) / restartShmemReq (:813-847) helpers
  // the L2 controller's call chains: processEx/ShReqFromL1Cache (:442-697),
  // processNullifyReq (:358-440), processNextReqFromL1Cache, with the
  // allocation's nullify run before the request continues (a stack of continuations)
  __device__ __forceinline__ void sh_run(SWork w, uint64_t& t)
  {
    SWork* stack = reinterpret_cast<SWork*>(sl.wstack);
    int sp = 0;
    for (;;) {
      if (failed) return;
      switch (w.kind) {
      case SW_PROC: {                             // getCacheLineInfo (:65-100)
        int32_t h = sh_evicted(w.addr);
        if (h != NO_ENT) { if (w.first) fail(); w.kind = SW_CONT; w.h = h; continue; }
        h = sh_slot(w.addr);
        L2.cnt(GG_CC_TAG_READS);
        const bool miss = h == NO_ENT;
        if (w.first) L2.miss_counters(w.addr, w.type == M_EX_REQ, miss);
        if (miss) {
          uint64_t ev = INV_ADDR;
          h = sh_allocate(w.addr, ev);
          if (h == NO_ENT) return;
          if (ev != INV_ADDR) {                   // a NULLIFY_REQ for the victim, queued and processed now (:162-182)
            qpush(ev, t, M_NULLIFY_REQ, tile);
            if (sp >= WSTACK) { fail(GG_DERR_CAP); return; }
            SWork c = w; c.kind = SW_CONT; c.h = h;
            stack[sp++] = c;
            w = SWork{ev, SW_NULL, 0, 0, 1, tile, 0};
            continue;
          }
        }
        w.kind = SW_CONT; w.h = h;
        continue;
      }
      case SW_CONT: {
        const int32_t h = w.h;
        const uint64_t a = w.addr;
        const uint32_t rq = w.req, cs = sh_cs(h), ds = sh_ds(h);
        bool done = false;
        if (cs == CS_DINV) {
          send(home(a), M_DRAM_FETCH_REQ, rq, a, t);               // fetchDataFromDram (:907-914)
        } else if (w.type == M_EX_REQ) {
          if (ds == DS_MODIFIED) {                                 // (MESI: EXCLUSIVE, the owner invalidated)
            send((uint32_t)e_owner(h), ME ? M_INV_REQ : M_FLUSH_REQ, rq, a, t);
          } else if (ds == DS_SHARED) {
            if (has(h, rq) && e_nsh(h) == 1) {                     // upgrade: the lone sharer
              set_owner(h, (int32_t)rq);
              sh_set_ds(h, DS_MODIFIED);
              send(rq, M_UPGRADE_REP, rq, a, t);
              done = true;
            } else {
              send_sharers(h, M_INV_REQ, rq, a, t);
            }
          } else {
            if (e_nsh(h) != 0) fail();
            add_sharer(h, rq);
            set_owner(h, (int32_t)rq);
            sh_set_ds(h, DS_MODIFIED);
            if (!w.data) L2.cnt(GG_CC_DATA_READS);                 // readCacheLine (:878-905)
            send(rq, M_EX_REP, rq, a, t);
            done = true;
          }
        } else {
          if (ds == DS_MODIFIED) {                                 // (MESI: DOWNGRADE_REQ to the exclusive owner)
            send((uint32_t)e_owner(h), ME ? M_DOWNGRADE_REQ : M_WB_REQ, rq, a, t);
          } else {
            uint32_t rep_type = M_SH_REP;
            if (ds == DS_UNCACHED) {
              if (e_nsh(h) != 0) fail();
              add_sharer(h, rq);
              if constexpr (ME) {                                  // …sh_l2_mesi/l2:671-687: an L1-D reader owns it EXCLUSIVE
                sh_set_ds(h, DS_MODIFIED);
                set_owner(h, (int32_t)rq);
                rep_type = M_SH_REP_EX;
              } else {
                sh_set_ds(h, DS_SHARED);
              }
            } else {
              add_sharer(h, rq);                                   // full map: always added
            }
            if (!w.data) L2.cnt(GG_CC_DATA_READS);
            send(rq, rep_type, rq, a, t);
            done = true;
          }
        }
        if (done) { sh_setinfo(h); w.kind = SW_NEXT; continue; }
        w.kind = SW_NONE;
        continue;
      }
      case SW_NULL: {                                              // the line in the evicted map
        const uint64_t a = w.addr;
        const int32_t h = sh_evicted(a);
        if (h == NO_ENT) { fail(); return; }
        const uint32_t cs = sh_cs(h), ds = sh_ds(h);
        if (ds == DS_MODIFIED) {
          send((uint32_t)e_owner(h), ME ? M_INV_REQ : M_FLUSH_REQ, w.req, a, t);
          w.kind = SW_NONE;
        } else if (ds == DS_SHARED) {
          send_sharers(h, M_INV_REQ, w.req, a, t);
          if (cs == CS_DIRTY && w.data) send(home(a), M_DRAM_STORE_REQ, w.req, a, t);
          w.kind = SW_NONE;
        } else {
          if (cs == CS_DIRTY && w.data) send(home(a), M_DRAM_STORE_REQ, w.req, a, t);
          dinvalidate(a);                                          // the entry deleted, the line out of the map
          w.kind = SW_NEXT;
        }
        continue;
      }
      case SW_NEXT: {
        t += P.gap_ps;                                     // Latency(1, L2 frequency)
        if (qcount(w.addr) < 1) { fail(); return; }
        qpop(w.addr);
        const int32_t f = qfront(w.addr);
        if (f < 0) { w.kind = SW_NONE; continue; }
        uint32_t type, req;
        front_update(f, t, type, req);
        if (type != M_EX_REQ && type != M_SH_REQ) { fail(); return; }
        w = SWork{w.addr, SW_PROC, type, 1, 0, req, 0};            // processShmemReq (:338-356)
        continue;
      }
      default:
        if (sp == 0) return;
        w = stack[--sp];
        continue;
      }
    }
  }
  // restartShmemReq (l2_cache_cntlr.cc:813-847): the front request of a, after a reply
  __device__ __forceinline__ void sh_restart(uint64_t a, int32_t f, int32_t h, uint32_t data, uint64_t& t)
  {
    t += P.gap_ps;                                     // Latency(1, L2 frequency)
    uint32_t type, req;
    front_update(f, t, type, req);
    const uint32_t ds = sh_ds(h);
    if (type == M_EX_REQ) { if (ds == DS_UNCACHED) sh_run(SWork{a, SW_PROC, type, 0, data, req, 0}, t); }
    else if (type == M_SH_REQ) sh_run(SWork{a, SW_PROC, type, 0, data, req, 0}, t);
    else if (type == M_NULLIFY_REQ) { if (ds == DS_UNCACHED) sh_run(SWork{a, SW_NULL, 0, 0, data, req, 0}, t); }
    else fail();
  }
  // L1CacheCntlr::insertCacheLine (l1_cache_cntlr.cc:230-274): an evicted line goes home
  __device__ __forceinline__ void sh_l1_insert(uint64_t a, uint32_t cs, uint64_t t)
  {
    bool ev; uint64_t ea = 0; uint32_t es = 0, el = 0;
    if (!L1.insert(a, cs, 0, ev, ea, es, el)) { fail(); return; }
    if (!ev) return;
    if (es == ST_M) send(home(ea), M_FLUSH_REP, tile, ea, t);
    else if (es == ST_S || (ME && es == ST_E)) send(home(ea), M_INV_REP, tile, ea, t);
    else fail();
  }
  // MESI: a hit rewrites the line's info, MODIFIED on a write
  // (operationPermissibleinL1Cache, …sh_l2_mesi/l1_cache_cntlr.cc:168-211)
  __device__ __forceinline__ void sh_mesi_hit(uint64_t a, bool wr, uint32_t cs)
  {
    if (!L1.set(a, wr ? (uint32_t)ST_M : cs, 0)) fail();
  }
  __device__ __forceinline__ bool sh_l1_ok(uint32_t cs, bool wr) const
  {
    return wr ? (cs == ST_M || (ME && cs == ST_E)) : cs != ST_I;
  }
  // invalidateCacheLine (:276-287)
  __device__ __forceinline__ void sh_l1_invalidate(uint64_t a)
  {
    uint32_t c, l;
    L1.get(a, c, l);
    if (!L1.set(a, ST_I, 0)) fail();
  }
  // processMemOpFromCore (l1_cache_cntlr.cc:80-144): no invalidate before a
  // miss; the request (handleMsgFromCore, :289-302, at once) to the line's home slice
  __device__ __forceinline__ void sh_app_access(uint64_t a, bool wr, uint64_t s)
  {
    uint64_t t = s;
    uint32_t cs, loc;
    L1.get(a, cs, loc);
    const bool hit = sh_l1_ok(cs, wr);
    if (ME && hit) sh_mesi_hit(a, wr, cs);
    L1.miss_counters(a, wr, !hit);
    if (hit) { t += P.lat_l1d; if (!L1.access(a, wr)) fail(); finish(s, t, GG_LVL_L1); return; }
    t += P.lat_l1t;
    if (out_addr != INV_ADDR) fail();
    out_addr = a; out_time = t;
    send(home(a), wr ? M_EX_REQ : M_SH_REQ, tile, a, t);
    blocked = 1;
    pend_start = s;
  }
  // MemoryManager::handleMsgFromNetwork (…sh_l2_msi/memory_manager.cc:215-294)
  __device__ __forceinline__ void sh_msg(const HMsg& m)
  {
    uint64_t t = m.arrival_ps;
    const uint64_t a = m.addr;
    const uint32_t ty = m.type;
    if (ty == M_EX_REP || ty == M_SH_REP || ty == M_UPGRADE_REP || (ME && ty == M_SH_REP_EX)) {   // handleMsgFromL2Cache (l1:304-409)
      if (!blocked || out_addr != a) { fail(); return; }
      if (ty == M_UPGRADE_REP) {
        uint32_t c1, l1;
        L1.get(a, c1, l1);
        if (c1 != ST_S) fail();
        if (!L1.set(a, ST_M, 0)) fail();
      } else {
        sh_l1_insert(a, ty == M_EX_REP ? (uint32_t)ST_M : ty == M_SH_REP_EX ? ST_E : (uint32_t)ST_S, t);
      }
      if (out_time > t) fail();
      t += P.lat_l1d;
      out_addr = INV_ADDR;
      const bool wr = (S.meta[rec] & GG_META_WRITE) != 0;             // access_num == 2 (l1:97-119)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      if (!sh_l1_ok(c1, wr)) { fail(); return; }
      if constexpr (ME) sh_mesi_hit(a, wr, c1);
      t += P.lat_l1d;
      if (!L1.access(a, wr)) fail();
      blocked = 0;
      finish(pend_start, t, GG_LVL_DIR);
    } else if (ME && ty == M_INV_REQ) {                               // …sh_l2_mesi/l1:432-498: a MODIFIED line is flushed
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      if (c1 == ST_M) {
        t += P.lat_l1d;
        if (!L1.access(a, false)) fail();                               // readCacheLine
        sh_l1_invalidate(a);
        send(m.src, M_FLUSH_REP, m.requester, a, t);
      } else {
        t += P.lat_l1t;
        if (c1 != ST_I) { sh_l1_invalidate(a); send(m.src, M_INV_REP, m.requester, a, t); }
      }
    } else if (ME && ty == M_DOWNGRADE_REQ) {                         // processDowngradeReqFromL2Cache (…sh_l2_mesi/l1:540-600)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      if (c1 != ST_I) {
        if (c1 == ST_M) {
          t += P.lat_l1d;
          if (!L1.access(a, false)) fail();
          send(m.src, M_WB_REP, m.requester, a, t);
        } else {
          if (c1 != ST_E) fail();
          t += P.lat_l1t;
          send(m.src, M_DOWNGRADE_REP, m.requester, a, t);
        }
        if (!L1.set(a, ST_S, 0)) fail();
      } else {
        t += P.lat_l1t;
      }
    } else if (ty == M_INV_REQ) {                                     // processInvReqFromL2Cache (l1:411-448)
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      t += P.lat_l1t;
      if (c1 != ST_I) {
        if (c1 != ST_S) fail();
        sh_l1_invalidate(a);
        send(m.src, M_INV_REP, m.requester, a, t);
      }
    } else if (ty == M_FLUSH_REQ || ty == M_WB_REQ) {                 // l1:450-536
      uint32_t c1, l1;
      L1.get(a, c1, l1);
      if (c1 != ST_I) {
        if (c1 != ST_M) fail();
        t += P.lat_l1d;
        if (!L1.access(a, false)) fail();                               // readCacheLine
        if (ty == M_FLUSH_REQ) { sh_l1_invalidate(a); send(m.src, M_FLUSH_REP, m.requester, a, t); }
        else { if (!L1.set(a, ST_S, 0)) fail(); send(m.src, M_WB_REP, m.requester, a, t); }
      } else {
        t += P.lat_l1t;
      }
    } else if (ty == M_EX_REQ || ty == M_SH_REQ) {                    // L2CacheCntlr::handleMsgFromL1Cache (l2:191-220)
      t += P.lat_l2d;
      qpush(a, t, ty, m.requester);
      if (qcount(a) == 1) sh_run(SWork{a, SW_PROC, ty, 1, 0, m.requester, 0}, t);
    } else if (ty == M_INV_REP || ty == M_FLUSH_REP || ty == M_WB_REP || (ME && ty == M_DOWNGRADE_REP)) {   // l2:222-270
      t += P.lat_l2d;
      int32_t h = sh_evicted(a);
      if (h == NO_ENT) { h = sh_slot(a); L2.cnt(GG_CC_TAG_READS); }
      if (h == NO_ENT) { fail(); return; }
      const uint32_t ds = sh_ds(h);
      if (ty == M_INV_REP) {                                          // processInvRepFromL1Cache (:699-729)
        if (ds == DS_SHARED) {
          remove_sharer(h, m.src);
          if (e_nsh(h) == 0) sh_set_ds(h, DS_UNCACHED);
        } else if (ME && ds == DS_MODIFIED) {                         // …sh_l2_mesi/l2:739-751: the exclusive owner
          if (e_nsh(h) != 1) fail();
          remove_sharer(h, m.src);
          set_owner(h, -1);
          sh_set_ds(h, DS_UNCACHED);
        }
      } else if (ME && ty == M_DOWNGRADE_REP) {                       // processDowngradeRepFromL1Cache (…sh_l2_mesi/l2:804-836)
        if (ds == DS_MODIFIED) { set_owner(h, -1); sh_set_ds(h, DS_SHARED); }
      } else if (ty == M_FLUSH_REP) {                                 // processFlushRepFromL1Cache (:731-773)
        if (ds == DS_MODIFIED) {
          const int32_t f = qfront(a);
          if (f < 0 || rq_get(f).type == M_SH_REQ) { if (h < 0) fail(); L2.cnt(GG_CC_DATA_WRITES); }   // writeCacheLine
          sh_set_cs(h, CS_DIRTY);
          remove_sharer(h, m.src);
          set_owner(h, -1);
          sh_set_ds(h, DS_UNCACHED);
        }
      } else {                                                        // processWbRepFromL1Cache (:775-811)
        if (ds == DS_MODIFIED) {
          if (h < 0) fail();
          L2.cnt(GG_CC_DATA_WRITES);
          sh_set_cs(h, CS_DIRTY);
          set_owner(h, -1);
          sh_set_ds(h, DS_SHARED);
        }
      }
      sh_setinfo(h);
      const int32_t f = qfront(a);
      if (f >= 0) sh_restart(a, f, h, ty != M_INV_REP && ty != M_DOWNGRADE_REP, t);
    } else if (ty == M_DRAM_FETCH_REP) {                              // L2CacheCntlr::handleMsgFromDram (l2:278-303)
      t += P.lat_l2d;
      const int32_t h = sh_slot(a);
      L2.cnt(GG_CC_TAG_READS);
      const int32_t f = qfront(a);
      if (h == NO_ENT || f < 0) { fail(); return; }
      const uint32_t ft = rq_get(f).type;
      if (ft == M_SH_REQ) L2.cnt(GG_CC_DATA_WRITES);                 // writeCacheLine
      else if (ft != M_EX_REQ) fail();
      sh_set_cs(h, CS_CLEAN);
      sh_setinfo(h);
      sh_restart(a, f, h, 1, t);
    } else if (ty == M_DRAM_FETCH_REQ) {                              // DramCntlr::handleMsgFromL2Cache (…sh_l2_msi/dram_cntlr.cc:19-52)
      t += dram_ps(t);
      send(m.src, M_DRAM_FETCH_REP, m.requester, a, t);
    } else if (ty == M_DRAM_STORE_REQ) {
      (void)dram_ps(t);
    } else {
      fail();
    }
  }

  __device__ __forceinline__ void flush()
  {
    {
      const uint32_t d2 = (uint32_t)__shfl((int)L2.cd, (int)((ln - GG_NUM_CACHE_COUNTERS) & 63u));
      const uint32_t d = ln < GG_NUM_CACHE_COUNTERS ? L1.cd : d2;
      if (ln < 2 * GG_NUM_CACHE_COUNTERS && d) S.cc[(size_t)lt * 2 * GG_NUM_CACHE_COUNTERS + ln] = ccv + d;
    }
    {
      const uint64_t d = sd;
      uint64_t* g = S.st + (size_t)lt * GG_NUM_TILE_STATS;
      if (ln == GG_CT_CLOCK_PS) { if (clk != p0.clk) g[ln] = clk; }
      else if (ln < GG_NUM_TILE_STATS && d) g[ln] = stv + d;
    }
    if (ln == 0) {
      if (rec != p0.rec) S.ts[lt].rec = rec;
      if (clk != p0.clk) S.ts[lt].clk = clk;
      if (pend_start != p0.pend_start) S.ts[lt].pend_start = pend_start;
      if (out_addr != p0.out_addr) S.ts[lt].out_addr = out_addr;
      if (out_time != p0.out_time) S.ts[lt].out_time = out_time;
      if (blocked != p0.blocked) S.ts[lt].blocked = blocked;
      if (seq != p0.seq) S.ts[lt].seq = seq;
      if (nrep != p0.nrep) S.ts[lt].nrep = nrep;
      if (nrq != p0.nrq) S.ts[lt].nrq = nrq;
    }
    if constexpr (MO) {
      if (ln < GG_NUM_PROTO_STATS && pd) S.ps[(size_t)lt * GG_NUM_PROTO_STATS + ln] += pd;
      if (ln == 0 && ncdl != ncdl0) S.ncdl[lt] = ncdl;
    }
  }
};

// ---------------------------------------------------------------------------
// ordering helpers (lane-parallel, O(n^2 / 64) compares; arrays in LDS or in
// the tile's global scratch, each phase closed by a workgroup barrier)
// ---------------------------------------------------------------------------
// The reference's per-channel FIFO merged by (arrival, sender): repeatedly the
// channel head with the least (arrival, sender).  That order is the sort by
// (P, sender, seq) with P = the largest arrival up to the message in its
// channel (a head can only leave after its channel's earlier messages, and
// every head waiting behind a larger arrival inherits it).  a = arrival,
// k = sender << 32 | seq; out = local indices in processing order.
__device__ __forceinline__ void order_inbox(uint32_t n, const uint64_t* a, const uint64_t* k, uint64_t* pm, uint32_t* out,
                                            uint32_t ln)
{
  for (uint32_t i = ln; i < n; i += 64) {
    const uint64_t ki = k[i];
    uint64_t m = 0;
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t kj = k[j];
      if ((kj >> 32) == (ki >> 32) && kj <= ki) m = max(m, a[j]);
    }
    pm[i] = m;
  }
  tsync();
  for (uint32_t i = ln; i < n; i += 64) {
    const uint64_t pi = pm[i], ki = k[i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) { const uint64_t pj = pm[j]; r += (pj < pi) || (pj == pi && k[j] < ki); }
    out[r] = i;                                   // the local index (its record: idx[i])
  }
  tsync();
}
// (time, send time, sender << 32 | seq) order: a port's service order (the
// canonical key of DESIGN.md §4)
__device__ __forceinline__ void order_port(uint32_t n, const uint64_t* t, const uint64_t* s, const uint64_t* k, const uint32_t* idx,
                           uint32_t* out, uint32_t ln)
{
  for (uint32_t i = ln; i < n; i += 64) {
    const uint64_t ti = t[i], si = s[i], ki = k[i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t tj = t[j], sj = s[j], kj = k[j];
      r += (tj < ti) || (tj == ti && (sj < si || (sj == si && kj < ki)));
    }
    out[r] = idx[i];
  }
  tsync();
}

// the same order, out[rank] = the entry's local index (its fields stay in
// the gathered arrays, no reload of the record)
__device__ __forceinline__ void order_port_local(uint32_t n, const uint64_t* t, const uint64_t* s, const uint64_t* k, uint32_t* out,
                                 uint32_t ln)
{
  for (uint32_t i = ln; i < n; i += 64) {
    const uint64_t ti = t[i], si = s[i], ki = k[i];
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) {
      const uint64_t tj = t[j], sj = s[j], kj = k[j];
      r += (tj < ti) || (tj == ti && (sj < si || (sj == si && kj < ki)));
    }
    out[r] = i;
  }
  tsync();
}

// Queue images (HQueue + max_size nodes, all 16-byte words) between HBM and
// LDS: image slot i of `img` (stride qimg bytes) <-> queue qi_of(i).  One
// flat index over every word of every image, 16 loads in flight per lane
// before their stores (a per-image copy waits one round trip per image).
template <bool IN, class QiOf, uint32_t U = 16>
__device__ __forceinline__ void imgs_copy(uint8_t* img, uint32_t qimg, uint32_t nimg, QiOf qi_of, HQueue* q, HNode* nd,
                                          uint32_t ms, uint32_t ln, uint32_t nl = 64)
{
  constexpr uint32_t HW = sizeof(HQueue) / 16;
  const uint32_t per = HW + ms, total = nimg * per;
  for (uint32_t j0 = 0; j0 < total; j0 += U * nl) {
    uint4 v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t j = j0 + u * nl + ln;
      v[u] = make_uint4(0, 0, 0, 0);
      if (j < total) {
        const uint32_t i = j / per, w = j % per;
        const uint64_t qi = qi_of(i);
        uint4* g = w < HW ? reinterpret_cast<uint4*>(q + qi) + w : reinterpret_cast<uint4*>(nd + qi * ms) + (w - HW);
        uint4* l = reinterpret_cast<uint4*>(img + (size_t)i * qimg) + w;
        v[u] = IN ? *g : *l;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t j = j0 + u * nl + ln;
      if (j >= total) continue;
      const uint32_t i = j / per, w = j % per;
      const uint64_t qi = qi_of(i);
      uint4* g = w < HW ? reinterpret_cast<uint4*>(q + qi) + w : reinterpret_cast<uint4*>(nd + qi * ms) + (w - HW);
      uint4* l = reinterpret_cast<uint4*>(img + (size_t)i * qimg) + w;
      if (IN) *l = v[u]; else *g = v[u];
    }
  }
}
__device__ __forceinline__ void img_in(uint8_t* img, HQueue* q, HNode* nd, uint32_t ms, uint32_t ln)
{
  imgs_copy<true>(img, 0, 1, [](uint32_t) { return (uint64_t)0; }, q, nd, ms, ln);
}
__device__ __forceinline__ void img_out(HQueue* q, HNode* nd, uint8_t* img, uint32_t ms, uint32_t ln)
{
  imgs_copy<false>(img, 0, 1, [](uint32_t) { return (uint64_t)0; }, q, nd, ms, ln);
}

// A router output port + link (RouterModel::processPacket router_model.cc:71-108,
// ElectricalLinkModel::processPacket electrical_link_model.cc:31-45): the
// port's queue delay, then router + link delay (zero-load part) and the
// counters {contention, router packets, buffer w+r (each), switch, crossbar,
// link}; done batch-wise by the walkers and k_c_step's SELF / injection ports.
__device__ __forceinline__ void net_ctr_add(uint64_t* ctr, uint32_t tile, const uint64_t* c)
{
  cadd(ctr, tile, GG_NC_ROUTER_CONTENTION_CYCLES, c[0]); cadd(ctr, tile, GG_NC_ROUTER_PACKETS, c[1]);
  cadd(ctr, tile, GG_NC_BUFFER_WRITES, c[2]); cadd(ctr, tile, GG_NC_BUFFER_READS, c[2]);
  cadd(ctr, tile, GG_NC_SWITCH_ALLOC, c[3]); cadd(ctr, tile, GG_NC_CROSSBAR, c[4]);
  cadd(ctr, tile, GG_NC_LINK_TRAVERSALS, c[5]);
}

// ---------------------------------------------------------------------------
// the step
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xy_stage_seg(const CP& P, const CS& S, uint32_t cur, uint32_t dst, bool& is_x)
{
  const uint32_t cx = cur % P.mw, cy = cur / P.mw, dx = dst % P.mw, dy = dst / P.mw;
  if (cx != dx) { is_x = true; return S.tseg[(size_t)cur * 2] * 2 + (dx > cx ? 1u : 0u); }
  is_x = false;
  return S.tseg[(size_t)cur * 2 + 1] * 2 + (dy > cy ? 1u : 0u);
}

__device__ __forceinline__ void import_one(const CP& P, const CS& S, const gg_cmsg& m, uint32_t* resumed);

// The end of a quantum in the device-driven loop (the launch after the step
// that sent nothing): every tile adds its status, the blocks deliver the held
// boundary records into the next quantum, and the last block to arrive picks
// the next quantum as gg_coherent_run / oracle_coh_run do (empty quanta
// skipped; blocked tiles with nothing in flight = deadlock).
__device__ __forceinline__ void quantum_end(const CP& P, const CS& S, uint32_t L, uint64_t q, uint64_t Q)
{
  const uint32_t ln = threadIdx.x, lt = blockIdx.x;
  volatile uint64_t* qs = S.qs;
  if (ln == 0) {
    const uint64_t r = S.ts[lt].rec;
    if (r < S.ts[lt].rec_end) {
      atomicAdd((unsigned long long*)&S.qs[QS_ACTIVE], 1ull);
      const uint32_t b = S.ts[lt].blocked;
      if (b == kBarWait) {
        atomicAdd((unsigned long long*)&S.qs[QS_BWAIT], 1ull);
        atomicMax((unsigned long long*)&S.qs[QS_BMAX], (unsigned long long)S.ts[lt].clk);
      } else if (b) atomicAdd((unsigned long long*)&S.qs[QS_BLOCKED], 1ull);
      else atomicMin((unsigned long long*)&S.qs[QS_MIN_NEXT],
                     (unsigned long long)(S.ts[lt].clk + rec_gap(S.meta[r]) * P.gap_ps));
    }
  }
  const uint32_t nb = *(volatile uint32_t*)S.bnd_cnt;
  for (uint32_t i = lt * 64 + ln; i < nb; i += gridDim.x * 64) import_one(P, S, S.bnd[i], &S.imp[(Q + 1) & 1]);
  __syncthreads();
  if (ln != 0) return;
  __threadfence();
  if (atomicAdd((unsigned long long*)&S.qs[QS_ARRIVED], 1ull) != gridDim.x - 1) return;
  __threadfence();
  const uint64_t active = qs[QS_ACTIVE], blocked = qs[QS_BLOCKED], mn = qs[QS_MIN_NEXT], qps = qs[QS_QPS];
  const uint64_t bw = qs[QS_BWAIT], bmax = qs[QS_BMAX];
  S.ri[GG_RI_QUANTA]++;
  S.ri[GG_RI_FINAL_QUANTUM] = q;
  uint64_t nq = q + 1, done = 0, rel = 0;
  if (active == 0 && nb == 0) done = 1;
  else if (nb == 0 && blocked == 0 && bw == active) {   // every unfinished tile waits at a barrier: release
    rel = bmax + 1;                                     // at the latest arrival, in the next quantum's step 0
    nq = max(q + 1, bmax / qps);
  }
  else if (nb == 0 && blocked == 0) nq = max(q + 1, mn / qps);
  else if (nb == 0) done = 2;                                          // blocked, nothing in flight: deadlock
  for (int i = 0; i < 4; ++i) S.ring[i] = 0;
  S.imp[Q & 1] = 0;
  *S.bnd_cnt = 0;
  qs[QS_ARRIVED] = 0; qs[QS_ACTIVE] = 0; qs[QS_BLOCKED] = 0; qs[QS_MIN_NEXT] = ~0ull;
  qs[QS_BWAIT] = 0; qs[QS_BMAX] = 0; qs[QS_REL] = rel;
  qs[QS_Q] = nq; qs[QS_START] = L + 1; qs[QS_COUNT] = Q + 1;
  qs[QS_DONE] = done;
  __threadfence();
}

// devloop: the quantum, its barrier and the step index come from S.qs (the
// quantum loop runs on the device, gg_coherent_run); otherwise the host
// drives one quantum (gg_coherent_quantum) and L is the step index.
// the tile's trace window: records wbase + lane (kept across the steps of a
// persistent launch; the records are read-only for the whole run)
struct TraceWin { uint64_t wbase, wa; uint32_t wm; };
constexpr uint64_t kNsFin = ~0ull, kNsBlk = ~0ull - 1;   // next start of a finished / blocked tile

template <bool LC, bool HR, bool F, int PR, class SL, class H>
__device__ __forceinline__ uint64_t tile_step(const CP& P, const CS& S, uint32_t lt, uint32_t k, uint32_t L, uint64_t barrier,
                                          TraceWin& W, SL& sl, uint8_t* clds, const TilePre& pre, const H& hk,
                                          uint32_t na, uint32_t ni, uint64_t rel);

// LC: cache state in LDS; HR: L1 hit runs (persistent small meshes, where
// long runs of hits between misses pay for the window look-up)
template <bool LC, bool HR, bool F = false, int PR = 0>
__device__ __forceinline__ void step_body(const CP& P, const CS& S, uint32_t L, uint32_t devloop, uint64_t barrier_arg,
                                          TraceWin& W)
{
  const uint32_t ln = threadIdx.x, lt = blockIdx.x;
  uint32_t k = L;
  uint64_t barrier = barrier_arg, q = 0, Q = 0;
  // one round trip: the launch state (written by earlier launches) spread
  // over lanes — lane i loads word i of the quantum state and of the step
  // ring, unconditionally, beside the tile's own state — then read out of
  // the lanes (per-word loads behind the devloop selects had compiled to a
  // chain of a load and a wait per word)
  static_assert(QS_N <= 64, "the quantum state fits a wave");
  const uint64_t qw = ln < QS_N ? S.qs[ln] : 0ull;
  const uint32_t rw = ln < 11 ? S.ring[ln] : 0u;              // ring[4], quiet, imp[2], live[4]
  TilePre pre;
  pre.load(S, lt, ln);
  uint64_t qsv[QS_N];
  uint32_t rv[11];
#pragma unroll
  for (int i = 0; i < QS_N; ++i) qsv[i] = devloop ? rl64(qw, (uint32_t)i) : 0ull;
#pragma unroll
  for (int i = 0; i < 11; ++i) rv[i] = rl32(rw, (uint32_t)i);
  if (devloop) {
    if (qsv[QS_DONE]) { if (lt == 0 && ln == 0) S.live[L & 3] = 0; return; }
    q = qsv[QS_Q]; Q = qsv[QS_COUNT];
    k = L - (uint32_t)qsv[QS_START];
    barrier = (q + 1) * qsv[QS_QPS];
  }
  const uint32_t p = k & 1u;
  if (k > 0) {
    if (!devloop && rv[4]) { if (lt == 0 && ln == 0) S.live[L & 3] = 0; return; }
    const uint32_t km = (k - 1) & 3;                  // selects, not a dynamically indexed (private) array
    const uint32_t sent = (km == 0 ? rv[0] : km == 1 ? rv[1] : km == 2 ? rv[2] : rv[3]) +
                          (k == 1 ? ((Q & 1) ? rv[6] : rv[5]) : 0u);
    if (sent == 0) {                                 // the previous step sent nothing: the quantum is done
      if (lt == 0 && ln == 0) { S.live[L & 3] = 0; if (!devloop) *S.quiet = k + 1; }   // (steps run + 1)
      if (devloop) quantum_end(P, S, L, q, Q);
      return;
    }
  }
  if (lt == 0 && ln == 0) {
    S.ri[GG_RI_STEPS]++; S.ring[(k + 2) & 3] = 0; S.npool[p ^ 1u] = P.L * kChunk;   // above the tiles' slices
    S.live[L & 3] = k + 1;
  }
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  StepLds& sl = *reinterpret_cast<StepLds*>(smem);
  const GHooks hk{P, S};
  const uint32_t na = P.net == GG_NET_EMESH_HOP_BY_HOP ? (p ? pre.narv1 : pre.narv0) : 0u;
  const uint32_t ni = p ? pre.ninb1 : pre.ninb0;
  tile_step<LC, HR, F, PR>(P, S, lt, k, L, barrier, W, sl, smem + P.cache_lds_off, pre, hk, na, ni,
                    devloop && k == 0 ? qsv[QS_REL] : 0ull);
}

// Publish of a hop-by-hop step whose sent records all fit the LDS sent list
// (Tile::put): self-sends to the next inbox (processCornerCases,
// network_model.cc:413-424); the rest through the tile's injection port
// (routePacket SEND_TILE, hop_by_hop.cc:151-159) in (send time, seq) order,
// then onto the X (or Y) run each enters.  Every field comes from LDS (the
// sent list, the tile's own run ids), and the port's queue is loaded while
// the list is sorted, so no record is read back from HBM.
template <class TT, class H>
__device__ __forceinline__ void publish_hbh_lds(TT& T, gg_cmsg* cur, uint32_t nloc, uint64_t& ri_net, uint64_t& ri_self,
                                                const H& hk, uint64_t& q1, uint64_t& q2, uint64_t& q3, uint64_t& q4)
{
  const CP& P = T.P; const CS& S = T.S;
  auto& sl = T.sl;
  const uint32_t ln = T.ln, lt = T.lt, tile = T.tile, p = T.p, seq0 = T.p0.seq;
  const uint32_t cx = tile % P.mw, cy = tile / P.mw;
  const uint64_t qi = (uint64_t)tile * 6 + P_INJ;
  HQueue* gq = S.nq + qi;
  HNode* gnd = S.nnd + qi * P.np.max_size;
  constexpr bool F = TT::kF;
  const bool regq = F ? P.np.qm != 0 : P.np.qm && P.np.qtype == GG_QM_HISTORY_TREE && P.np.max_size <= kQMax;
  const bool wave = !F && P.np.qm && P.np.max_size <= kQMax && !regq;
  RegQueue rq;
  RegQueue::Raw rqr;                                  // (issued with the sends' list atomics, read after the order)
  uint32_t nn = 0;
  bool rq_loaded = false;
  // The list slots (inbox of the next step for self-sends, the X / Y run
  // for the rest) do not depend on the port: the slot atomics of the first 64
  // sends are issued here and their list words stored after the port's
  // requests, so their round trip overlaps the ordering and the requests
  // (a list's order is free: the walkers and the inbox order by the keys)
  uint32_t* late_p = nullptr;                        // an inbox list (self-send) ...
  uint64_t* late_q = nullptr;                        // ... or a run list
  uint32_t late_j = ~0u, late_r = 0, late_cap = 0;   // the raw atomic result, checked at the store
  uint64_t late_v = 0;
  for (uint32_t i0 = 0; i0 < nloc; i0 += 64) {
    const uint32_t i = i0 + ln;
    uint64_t e = 0, ts = 0;
    bool self = false, net = false;
    if (i < nloc) { e = sl.x3[i]; ts = sl.x4[i]; self = (uint32_t)((e >> 32) & 0x3FFFFFFFu) == tile; net = !self; }
    const uint32_t r = (uint32_t)e;
    if (self) {
      uint32_t* lp = inb(S, p ^ 1u) + (size_t)lt * P.IC;
      const uint32_t j = atomicAdd(ninb_at(S, p ^ 1u, lt), 1u);     // (hk.inbox_slot, checked at the store)
      if (i0 == 0) { late_p = lp; late_j = j; late_r = r; late_cap = P.IC; }
      else if (j >= P.IC) atomicOr(S.err, GG_DERR_CAP);
      else lp[j] = r;
      ri_self++;
    }
    const uint64_t m = __ballot(net);
    if (m && regq && !rq_loaded) { rqr = RegQueue::issue(gq, gnd, P.np.max_size, ln); rq_loaded = true; }
    const uint32_t pos = nn + (uint32_t)__builtin_popcountll(m & ((1ull << ln) - 1));
    if (net) {
      const uint32_t d = (uint32_t)((e >> 32) & 0x3FFFFFFFu), dx = d % P.mw, dy = d / P.mw;
      const bool is_x = cx != dx;
      const uint32_t sg = is_x ? T.p0.segx * 2 + (dx > cx ? 1u : 0u) : T.p0.segy * 2 + (dy > cy ? 1u : 0u);
      const uint64_t lc = e >> 62;                        // length class
      sl.x1[pos] = ts;
      sl.x2[pos] = ((uint64_t)(seq0 + i) << 2) | lc;      // the sender is this tile: its seq orders equal times
      sl.i1[pos] = r;
      sl.x4[pos] = lc << 32;                              // (read above for slot i >= pos, in program order)
      // onto the X (or Y) run the packet enters (hk.seg_slot, checked at the store)
      const uint32_t j = atomicAdd(&(is_x ? S.nxl : S.nyl)[sg], 1u);
      uint64_t* lp = (is_x ? S.xl : S.yl) + (size_t)sg * P.seg_cap;
      const uint64_t v = (uint64_t)r | ((uint64_t)d << 32);
      if (i0 == 0) { late_q = lp; late_j = j; late_v = v; late_cap = P.seg_cap; }
      else if (j >= P.seg_cap) atomicOr(S.err, GG_DERR_CAP);
      else lp[j] = v;
      ri_net++;
    }
    nn += (uint32_t)__builtin_popcountll(m);
  }
  tsync();
  auto late_store = [&]() {                              // the list words of the first 64 sends
    if (late_p) { if (late_j >= late_cap) atomicOr(S.err, GG_DERR_CAP); else late_p[late_j] = late_r; }
    if (late_q) { if (late_j >= late_cap) atomicOr(S.err, GG_DERR_CAP); else late_q[late_j] = late_v; }
  };
  if (!nn) { late_store(); return; }
  if (DG(S.trs)) q1 = __builtin_amdgcn_s_memtime();
  order_port_local(nn, sl.x1, sl.x1, sl.x2, sl.i2, ln);
  if (DG(S.trs)) q2 = __builtin_amdgcn_s_memtime();
  // the port's queue: tr in HBM, trl the LDS image (one address space each:
  // a pointer merged from the two would make every queue access flat)
  HTree tr{gq, gnd, 1, P.np.analytical != 0};
  HTree trl{reinterpret_cast<HQueue*>(sl.pimg), reinterpret_cast<HNode*>(sl.pimg + sizeof(HQueue)), 1,
            P.np.analytical != 0};
  if (wave) {
    img_in(sl.pimg, gq, gnd, P.np.max_size, ln);
    tsync();
  }
  if (regq) rq.finish(rqr, gq, gnd, 1, P.np.analytical != 0, ln);
  if (DG(S.trs)) { (void)__builtin_amdgcn_readfirstlane((int)rq.a0); q3 = __builtin_amdgcn_s_memtime(); }
  uint64_t ps = 0, fs = 0, bs = 0;
  for (uint32_t c0 = 0; c0 < nn; c0 += 64) {
    const uint32_t cnt = min(64u, nn - c0);
    uint32_t r = 0, nf_ = 0, bits = 0;
    uint64_t sp = 0;
    if (ln < cnt) {
      const uint32_t e = sl.i2[c0 + ln];
      r = sl.i1[e];
      sp = sl.x1[e];
      bits = class_bits(P, (uint32_t)(sl.x4[e] >> 32));
      nf_ = (uint32_t)nflits(P.np, bits);
    }
    uint64_t oq = 0;
    for (uint32_t k = 0; k < cnt; ++k) {
      const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)nf_, (int)k);
      uint64_t qd = 0;
      if (P.np.qm) {
        const uint64_t tc = time_to_cycles(rl64(sp, k), P.np.f);
        if constexpr (F) qd = rq.request(tc, nf, S.err); else qd = regq ? rq.request(tc, nf, S.err) : (wave ? trl.delay_w(tc, nf, S.err, ln) : tr.delay(tc, nf, S.err));
      }
      if (ln == k) oq = qd;
      fs += nf; bs += (uint32_t)__builtin_amdgcn_readlane((int)bits, (int)k);   // updateSendCounters (network_model.cc:228-251)
    }
    ps += cnt;
    if (ln < cnt) {
      gg_cmsg* g = cur + r;
      g->arrival_ps = sp + lat_to_ps(0, P.np.f) + lat_to_ps(oq, P.np.f);
      g->zero_load_ps = 0;
      g->hop = tile;
    }
  }
  if (DG(S.trs)) q4 = __builtin_amdgcn_s_memtime();
  if (regq) rq.store(gq, gnd);
  if (wave) { tsync(); img_out(gq, gnd, sl.pimg, P.np.max_size, ln); }
  if (ln == 0) {
    cadd(S.ctr, tile, GG_NC_PACKETS_SENT, ps); cadd(S.ctr, tile, GG_NC_FLITS_SENT, fs);
    cadd(S.ctr, tile, GG_NC_BITS_SENT, bs);
  }
  late_store();
  tsync();
}

// One tile's step k (parity k & 1) of the quantum that ends at `barrier`, on
// the calling wave: the SELF port + receive of the packets that
// reached the tile (na), the inbox (ni records), the trace, publish, write
// back.  Deliveries go through the hooks.
template <bool LC, bool HR, bool F, int PR, class SL, class H>
__device__ __forceinline__ uint64_t tile_step(const CP& P, const CS& S, uint32_t lt, uint32_t k, uint32_t L, uint64_t barrier,
                                          TraceWin& W, SL& sl, uint8_t* clds, const TilePre& pre, const H& hk,
                                          uint32_t na, uint32_t ni, uint64_t rel)
{
  const uint32_t ln = lane_id(), p = k & 1u;
  PROF_T0();
  constexpr bool MO = PR == 1, SH = PR >= 2;   // (PR 2 / 3: the shared-L2 MSI / MESI controllers)
  Tile<SL, H, F, PR> T(P, S, lt, p, sl, hk, clds, std::integral_constant<bool, LC>(), pre);
  T.tr_on = DG(S.trs) != nullptr && L < S.tr_n;
  const gg_cmsg* prev = pool(S, p ^ 1u);     // records delivered to this step
  uint64_t* gscr = S.gscr + (size_t)lt * 6 * P.IC;
  // NoC counters of the SELF port (lanes 0-6) and of the receiver
  // (lanes 8-12: packets, flits, bits received, latency, contention)
  uint64_t ncd = 0;

  // ---- 0. hop-by-hop: SELF output port + receive of last step's packets (routePacket
  // at the receiver, hop_by_hop.cc:223-256; __processReceivedPacket, network_model.cc:118-150)
  PROF_AT(_sa);
  uint64_t _sb = 0, _sc = 0, _sd = 0, _se = 0, _sf = 0, _q1 = 0, _q2 = 0, _q3 = 0, _q4 = 0, _q1b = 0;
  uint64_t _hd = 0, _hl = 0, _hn = 0;                          // trace: handler cycles (directory / L2), counts
  // The directory request FIFO (<= 64 entries) and the DRAM queue image are
  // loaded now, in the same round as the SELF batch's loads, held in
  // registers across the SELF phase and written to LDS after it (loaded
  // after the SELF phase they would cost the inbox a round trip of their own)
  const uint32_t n = ni + na;
  const bool rq_fit = T.nrq + 2 * n + 2 <= SL::kRq, pre_rq = rq_fit && T.nrq <= 64;
  const bool dq_fit = P.dram_qm && P.max_list <= kQMax && n;
  constexpr uint32_t kHW = sizeof(HQueue) / 16;
  static_assert(kHW + kQMax <= 3 * 64, "the DRAM image prefetch holds 3 words per lane");
  uint64_t fq[3];
  uint4 dv[3];
  if (pre_rq) {
    const uint64_t* g = reinterpret_cast<const uint64_t*>(S.rq + (size_t)lt * P.QC);   // 3 words per entry
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) { const uint32_t j = ln + 64 * u; fq[u] = j < 3 * T.nrq ? g[j] : 0ull; }
  }
  if (dq_fit) {
    const uint4* gq_ = reinterpret_cast<const uint4*>(S.dq + lt);
    const uint4* gn_ = reinterpret_cast<const uint4*>(S.dnd + (size_t)lt * P.max_list);
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) {
      const uint32_t j = ln + 64 * u;
      dv[u] = j < kHW ? gq_[j] : j < kHW + P.max_list ? gn_[j - kHW] : make_uint4(0, 0, 0, 0);
    }
  }
  // SELF arrivals with no other inbox records: the SELF batch leaves the
  // inbox keys (new arrival, sender << 32 | seq, record) in LDS, so the inbox
  // is ordered without gathering its records again
  const bool self_keys = ni == 0 && na && na <= SL::kIn;
  uint64_t h_addr = 0;                           // address and type | requester << 8 of the message at local index lane
  uint32_t h_tr = 0;
  if (na) {
    if (DG(S.prof) || DG(S.trs)) _sb = __builtin_amdgcn_s_memtime();
    const uint32_t* al = arv(S, p) + (size_t)lt * P.IC;
    // the port's queue in registers for the batch (RegQueue, its loads in
    // flight beside the records'); other models on an LDS image
    const uint64_t qi = (uint64_t)T.tile * 6 + P_SELF;
    HQueue* gq = S.nq + qi;
    HNode* gnd = S.nnd + qi * P.np.max_size;
    const bool regq = F ? P.np.qm != 0 : P.np.qm && P.np.qtype == GG_QM_HISTORY_TREE && P.np.max_size <= kQMax;
    const bool wave = !F && P.np.qm && P.np.max_size <= kQMax && !regq;
    // (its loads issued now, beside the batch's list words; read after the order)
    RegQueue rq;
    RegQueue::Raw rqr;
    if (regq) rqr = RegQueue::issue(gq, gnd, P.np.max_size, ln);
    const uint64_t zps = lat_to_ps((uint64_t)P.np.router_delay + P.np.link_delay, P.np.f);
    uint64_t cq = 0, cf = 0;                                   // uniform: contention cycles, flits
    uint64_t rf = 0, rb = 0, rl = 0, rc = 0;                   // uniform: received flits, bits, latency, contention
    const uint64_t rn = na;
    gg_cmsg* pv = const_cast<gg_cmsg*>(prev);
    // the batch in LDS (or, past kIn entries, in HBM scratch): one instance
    // per place, so every access has one address space (no flat accesses)
    auto self_batch = [&](auto in_lds) __attribute__((always_inline)) {
    constexpr bool LD = decltype(in_lds)::value;
    uint64_t* t_ = LD ? sl.x1 : gscr; uint64_t* s_ = LD ? sl.x2 : gscr + P.IC; uint64_t* k_ = LD ? sl.x3 : gscr + 2 * P.IC;
    uint64_t* z_a = LD ? sl.x4 : gscr + 5 * P.IC;
    uint32_t* i_ = LD ? sl.i1 : (uint32_t*)(gscr + 3 * P.IC); uint32_t* o_ = LD ? sl.i2 : (uint32_t*)(gscr + 4 * P.IC);
    // 4 records per lane in flight: the list words, then the records (a
    // fan-in of hundreds of acknowledgements at a hot line's home otherwise
    // waits two dependent memory round trips per 64 records); every field
    // the port and the receiver need goes to LDS (key bit 0: has data)
    for (uint32_t i0 = ln; i0 < na; i0 += 256) {
      uint32_t rr[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) rr[u] = i0 + 64 * u < na ? al[i0 + 64 * u] : 0u;
      uint64_t ta[4], sa[4], za[4];
      uint32_t sr[4], sq[4], ty[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i0 + 64 * u < na) {
          const gg_cmsg& m = prev[rr[u]];
          ta[u] = m.arrival_ps; sa[u] = m.send_ps; za[u] = m.zero_load_ps; sr[u] = m.src; sq[u] = m.seq; ty[u] = m.type;
          if (u == 0 && i0 == ln) { h_addr = m.addr; h_tr = m.type | (m.requester << 8); }   // the handler's fields
        }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = i0 + 64 * u;
        if (i < na) {
          t_[i] = ta[u]; s_[i] = sa[u]; z_a[i] = za[u]; i_[i] = rr[u];
          k_[i] = ((uint64_t)sr[u] << 34) | ((uint64_t)sq[u] << 2) | len_class(ty[u]);
        }
      }
    }
    tsync();
    if (DG(S.prof) || DG(S.trs)) _sc = __builtin_amdgcn_s_memtime();
    order_port_local(na, t_, s_, k_, o_, ln);
    if (DG(S.prof) || DG(S.trs)) _sd = __builtin_amdgcn_s_memtime();
    // the port's queue: tr in HBM, trl the LDS image (one address space each:
    // a pointer merged from the two would make every queue access flat)
    HTree tr{gq, gnd, 1, P.np.analytical != 0};
    HTree trl{reinterpret_cast<HQueue*>(sl.pimg), reinterpret_cast<HNode*>(sl.pimg + sizeof(HQueue)), 1,
              P.np.analytical != 0};
    if (wave) {
      img_in(sl.pimg, gq, gnd, P.np.max_size, ln);
      tsync();
    }
    if (regq) rq.finish(rqr, gq, gnd, 1, P.np.analytical != 0, ln);
    if (DG(S.prof) || DG(S.trs)) { (void)__builtin_amdgcn_readfirstlane((int)rq.a0); _se = __builtin_amdgcn_s_memtime(); }
    for (uint32_t c0 = 0; c0 < na; c0 += 64) {
      const uint32_t cnt = min(64u, na - c0);
      uint32_t r = 0, nf_ = 0, bits = 0, e = 0;
      uint64_t tv = 0, z_ = 0, sp = 0;
      if (ln < cnt) {
        e = o_[c0 + ln];                                         // local index of the packet of rank c0 + ln
        r = i_[e];
        tv = t_[e]; z_ = z_a[e]; sp = s_[e];
        bits = class_bits(P, (uint32_t)(k_[e] & 3u));
        nf_ = (uint32_t)nflits(P.np, bits);
      }
      uint64_t ot = tv, oz = z_;
      const uint64_t x0 = DG(S.prof) && regq ? rq.A(rq.sz - 1) : 0;
      uint32_t ntail = 0;
      for (uint32_t k = 0; k < cnt; ++k) {
        const uint64_t t = rl64(tv, k);
        const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)nf_, (int)k);
        uint64_t qd = 0;
        if (P.np.qm) {
          const uint64_t tc = time_to_cycles(t, P.np.f);
          ntail += tc >= x0;
          if constexpr (F) qd = rq.request(tc, nf, S.err); else qd = regq ? rq.request(tc, nf, S.err) : (wave ? trl.delay_w(tc, nf, S.err, ln) : tr.delay(tc, nf, S.err));
        }
        cq += qd; cf += nf;
        // serialization + receive (network_model.cc:118-150), uniform: the
        // lane of packet k keeps its new arrival / zero-load for the store
        const uint64_t ser = lat_to_ps(nf, P.np.f);
        const uint64_t t2 = t + zps + lat_to_ps(qd, P.np.f) + ser, z2 = rl64(z_, k) + zps + ser;
        const uint64_t ct = t2 - rl64(sp, k) - z2;
        rf += nf; rb += (uint32_t)__builtin_amdgcn_readlane((int)bits, (int)k); rl += z2 + ct; rc += ct;
        if (ln == k) { ot = t2; oz = z2; }
      }
      if (DG(S.prof) && ln == 0) prof_batch(S, 0, cnt, ntail);
      if (DG(S.trs)) _sf = __builtin_amdgcn_s_memtime();
      if (ln < cnt) {
        pv[r].arrival_ps = ot; pv[r].zero_load_ps = oz;
        if (LD && self_keys) { const uint64_t kk = k_[e]; t_[e] = ot; s_[e] = ((kk >> 34) << 32) | ((kk >> 2) & 0xFFFFFFFFull); }
      }
    }
    };
    if (na <= SL::kIn) self_batch(std::true_type{}); else self_batch(std::false_type{});
    if (regq) rq.store(gq, gnd);
    if (wave) { tsync(); img_out(gq, gnd, sl.pimg, P.np.max_size, ln); }
    // lanes 0-6: the SELF port (contention, router packets, buffer writes, switch, crossbar, link, buffer reads), 8-12: the receiver
    ncd = ln == 0 ? (P.np.qm ? cq : 0ull) : ln == 1 ? (P.np.qm ? (uint64_t)na : 0ull) : ln == 3 ? (uint64_t)na
        : (ln == 2 || ln == 4 || ln == 5 || ln == 6) ? cf : ln == 8 ? rn : ln == 9 ? rf : ln == 10 ? rb
        : ln == 11 ? rl : ln == 12 ? rc : 0ull;
    hk.clear_arv(p, lt);
    tsync();
  }

  PROF_AT(_p1);
  if (DG(S.prof) && ln == 0 && na) {
    atomicAdd(&DG(S.prof)[90], (unsigned long long)(_sa - _p0)); atomicAdd(&DG(S.prof)[91], (unsigned long long)(_sb - _sa));
    atomicAdd(&DG(S.prof)[92], (unsigned long long)(_sc - _sb)); atomicAdd(&DG(S.prof)[93], (unsigned long long)(_sd - _sc));
    atomicAdd(&DG(S.prof)[94], (unsigned long long)(_se - _sd)); atomicAdd(&DG(S.prof)[95], (unsigned long long)(_p1 - _se));
    atomicAdd(&DG(S.prof)[96], 1ull);
  }
  if (DG(S.prof) && ln == 0 && !na) { atomicAdd(&DG(S.prof)[97], (unsigned long long)(_sa - _p0)); atomicAdd(&DG(S.prof)[98], 1ull); }
  // directory request FIFO in LDS when it cannot outgrow it this step
  if (rq_fit) {
    if (pre_rq) {
      GG_LDS uint64_t* l = reinterpret_cast<GG_LDS uint64_t*>(T.lrq());
#pragma unroll
      for (uint32_t u = 0; u < 3; ++u) { const uint32_t j = ln + 64 * u; if (j < 3 * T.nrq) l[j] = fq[u]; }
    } else {
      const CReq* g = S.rq + (size_t)lt * P.QC;
      for (uint32_t i = ln; i < T.nrq; i += 64) sl.rq[i] = g[i];
    }
    T.rq_lds = true;
  }
  if (dq_fit) {
    uint4* l = reinterpret_cast<uint4*>(sl.dimg);
#pragma unroll
    for (uint32_t u = 0; u < 3; ++u) { const uint32_t j = ln + 64 * u; if (j < kHW + P.max_list) l[j] = dv[u]; }
    T.dq_lds = true;
  }
  tsync();
  if (n) {
    const bool lds = n <= SL::kIn;
    const uint32_t* il = inb(S, p) + (size_t)lt * P.IC;
    const uint32_t* al = arv(S, p) + (size_t)lt * P.IC;
    // gather + order: one instance per place of the batch (as self_batch)
    auto inbox_batch = [&](auto in_lds) __attribute__((always_inline)) {
    constexpr bool LD = decltype(in_lds)::value;
    uint64_t* a_ = LD ? sl.x1 : gscr; uint64_t* k_ = LD ? sl.x2 : gscr + P.IC; uint64_t* m_ = LD ? sl.x3 : gscr + 2 * P.IC;
    uint32_t* i_ = LD ? sl.i1 : (uint32_t*)(gscr + 3 * P.IC); uint32_t* o_ = LD ? sl.i2 : (uint32_t*)(gscr + 4 * P.IC);
    for (uint32_t i0 = ln; i0 < n && !(LD && self_keys); i0 += 256) {   // 4 records per lane in flight
      uint32_t rr[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = i0 + 64 * u;
        rr[u] = i < n ? (i < ni ? il[i] : al[i - ni]) : 0u;
      }
      uint64_t ta[4];
      uint32_t sr[4], sq[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i0 + 64 * u < n) {
          const gg_cmsg& m = prev[rr[u]];
          ta[u] = m.arrival_ps; sr[u] = m.src; sq[u] = m.seq;
          if (u == 0 && i0 == ln) { h_addr = m.addr; h_tr = m.type | (m.requester << 8); }   // the handler's fields
        }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t i = i0 + 64 * u;
        if (i < n) { a_[i] = ta[u]; k_[i] = ((uint64_t)sr[u] << 32) | sq[u]; i_[i] = rr[u]; }
      }
    }
    tsync();
    hk.clear_inb(p, lt);
    order_inbox(n, a_, k_, m_, o_, ln);
    };
    if (lds) inbox_batch(std::true_type{}); else inbox_batch(std::false_type{});
    const uint32_t* go_ = (const uint32_t*)(gscr + 4 * P.IC);
    const uint32_t* gi_ = (const uint32_t*)(gscr + 3 * P.IC);
    PROF_AT(_p1b);
    _q1b = _p1b;
    if (DG(S.prof) && ln == 0) atomicAdd(&DG(S.prof)[9], (unsigned long long)(_p1b - _p1));
    for (uint32_t j = 0; j < n && !T.failed; ++j) {
      // the message: arrival and sender from the ordering arrays, address /
      // type / requester from the gather's registers (local index < 64: no
      // reload of the record), else from the record
      HMsg m;
      if (lds) {
        const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)sl.i2[j]);
        m.arrival_ps = sl.x1[e]; m.src = (uint32_t)(sl.x2[e] >> 32);
        if (e < 64) {
          m.addr = rl64(h_addr, e);
          const uint32_t tr = rl32(h_tr, e);
          m.type = tr & 0xFFu; m.requester = tr >> 8;
        } else {
          const gg_cmsg& g = prev[sl.i1[e]];
          m.addr = g.addr; m.type = g.type; m.requester = g.requester;
        }
        m.single_rx = MO && m.type == M_IFC_REQ ? prev[sl.i1[e]].single_rx : 0u;
      } else {
        const gg_cmsg& g = prev[gi_[go_[j]]];
        m.arrival_ps = g.arrival_ps; m.src = g.src; m.addr = g.addr; m.type = g.type; m.requester = g.requester;
        m.single_rx = MO ? g.single_rx : 0u;
      }
      T.stat(GG_CT_MSGS_RECEIVED, 1);
      const uint64_t h0 = DG(S.trs) ? __builtin_amdgcn_s_memtime() : 0;
      const bool dm = to_directory(m.type);
      if constexpr (SH) T.sh_msg(m);
      else if constexpr (MO) { if (dm) T.directory_msg_mo(m); else T.l2_msg_mo(m); }
      else { if (dm) T.directory_msg(m); else T.l2_msg(m); }
      if (DG(S.trs)) {
        const uint64_t h1 = __builtin_amdgcn_s_memtime();
        if (dm) { _hd += h1 - h0; _hn += 1; } else { _hl += h1 - h0; _hn += 1ull << 32; }
      }
    }
  }

  PROF_AT(_p2);
  // a barrier released at the quantum boundary: continue at the latest
  // arrival (the SyncInstruction of sync_client.cc:308-314 is the stall)
  if (rel && T.blocked == kBarWait) {
    const uint64_t t = rel - 1;
    if (S.out && ln == 0) S.out[T.rec] = ((t - T.clk) << 2) | GG_LVL_SYNC;
    T.clk = t; ++T.rec; T.blocked = 0;
  }
  // ---- 2. the trace (records fetched 64 at a time, one per lane)
  {
    const uint64_t line_mask = ~((1ull << P.log_line) - 1);
    uint64_t wbase = W.wbase, wa = W.wa;
    uint32_t wm = W.wm;
    uint64_t stop = ~0ull;
    while (!T.blocked && !T.failed) {
      const uint64_t r = T.rec;
      if (r >= T.rec_end) break;
      if (wbase == ~0ull || r >= wbase + 64) {
        wbase = r;
        wa = 0; wm = 0;
        if (r + ln < T.rec_end) { wa = S.addr[r + ln]; wm = S.meta[r + ln]; }
      }
      const int o = (int)(r - wbase);
      // a run that ended inside the window ended on a record that is not a
      // plain L1 hit before the barrier: that one goes straight to app_access
      // hit runs pay a window look-up: start one only on a record that hits
      bool try_run = HR && r != stop && !P.no_hit_runs;
      if (try_run) {
        const uint32_t m0 = rl32(wm, (uint32_t)o);
        const uint32_t cs = T.L1.probe(rl64(wa, (uint32_t)o) & line_mask);
        try_run = (m0 & GG_META_WRITE) ? cs == ST_M : cs != ST_I;
      }
      if (try_run) {
        PROF_AT(_h0);
        if (DG(S.prof) && ln == 0) atomicAdd(&DG(S.prof)[39], (unsigned long long)_h0);
        const uint32_t nh = T.l1_hit_run(wbase, (uint32_t)o, wa, wm, line_mask, barrier);
        PROF_AT(_h1);
        if (DG(S.prof) && ln == 0) { atomicAdd(&DG(S.prof)[33], (unsigned long long)(_h1 - _h0)); atomicAdd(&DG(S.prof)[34], (unsigned long long)nh); }
        if (nh) { if (o + nh < 64) stop = T.rec; continue; }
      }
      PROF_AT(_ha);
      const uint32_t meta = rl32(wm, (uint32_t)o);
      if (meta == GG_META_BARRIER) {                                 // CarbonBarrierWait at the tile's clock
        if (T.clk < barrier) T.blocked = kBarWait;
        break;
      }
      const uint64_t s = T.clk + (uint64_t)((meta & 0x7FFFFFFFu) >> 1) * P.gap_ps;
      if (s >= barrier && !(meta & GG_META_CONT)) break;             // a multi-line access is one instruction
      T.app_access(rl64(wa, (uint32_t)o) & line_mask, (meta & GG_META_WRITE) != 0, s);
      PROF_AT(_h2);
      if (DG(S.prof) && ln == 0) { atomicAdd(&DG(S.prof)[35], (unsigned long long)(_h2 - _ha)); atomicAdd(&DG(S.prof)[36], 1ull); }
    }
    W.wbase = wbase; W.wa = wa; W.wm = wm;
  }

  PROF_AT(_p3);
  // ---- 3. publish this step's records
  if (T.nch) sl.ch[2 * (T.nch - 1) + 1] = T.cused;
  tsync();
  gg_cmsg* cur = pool(S, p);
  const uint32_t np_ = T.nsent;
  uint64_t ri_net = 0, ri_self = 0, ri_bnd = 0;
  if (np_) {
    // one instance per place of the batch (as self_batch)
    auto pub_batch = [&](auto in_lds) __attribute__((always_inline)) {
    constexpr bool LD = decltype(in_lds)::value;
    uint64_t* t_ = LD ? sl.x1 : gscr; uint64_t* s_ = LD ? sl.x2 : gscr + P.IC; uint64_t* k_ = LD ? sl.x3 : gscr + 2 * P.IC;
    uint32_t* i_ = LD ? sl.i1 : (uint32_t*)(gscr + 3 * P.IC); uint32_t* o_ = LD ? sl.i2 : (uint32_t*)(gscr + 4 * P.IC);
    if (!LD && np_ > P.IC) T.fail(GG_DERR_CAP);
    // the records of the chunks, in allocation order
    uint32_t off = 0;
    for (uint32_t c = 0; c < T.nch && !T.failed; ++c) {
      const uint32_t b = sl.ch[2 * c], u = sl.ch[2 * c + 1];
      for (uint32_t r = ln; r < u; r += 64) i_[off + r] = b + r;
      off += u;
    }
    tsync();
    const uint32_t nloc = T.failed ? 0u : off;
    if (P.net != GG_NET_EMESH_HOP_BY_HOP) {
      // NetworkModel::routePacket closed form (hop counter / magic) + delivery
      for (uint32_t i = ln; i < nloc; i += 64) {
        const uint32_t r = i_[i];
        gg_cmsg m = cur[r];
        uint64_t zl;
        m.arrival_ps = route_closed_form(P.np, m.src, m.dst, msg_bits(P, m.type), m.send_ps,
                                         zl, S.ctr);
        m.zero_load_ps = zl;
        if (m.src == m.dst) ri_self++; else ri_net++;
        if (S.shard[m.src] == S.shard[m.dst]) {
          const int32_t ld = S.ltile[m.dst];
          const uint32_t j = hk.inbox_slot(p ^ 1u, (uint32_t)ld);
          if (j == ~0u) { atomicOr(S.err, GG_DERR_CAP); continue; }
          cur[r].arrival_ps = m.arrival_ps; cur[r].zero_load_ps = zl;
          inb(S, p ^ 1u)[(size_t)ld * P.IC + j] = r;
        } else {
          if (!hk.bnd_put(m)) { atomicOr(S.err, GG_DERR_CAP); continue; }
          ri_bnd++;
        }
      }
    } else if (LD && np_ == nloc) {
      publish_hbh_lds(T, cur, nloc, ri_net, ri_self, hk, _q1, _q2, _q3, _q4);
    } else {
      // self-sends: straight to the next inbox (processCornerCases, network_model.cc:413-424)
      uint32_t nn = 0;
      for (uint32_t i0 = 0; i0 < nloc; i0 += 64) {
        const uint32_t i = i0 + ln;
        bool self = false, net = false;
        uint32_t r = 0;
        if (i < nloc) { r = i_[i]; self = cur[r].dst == T.tile; net = !self; }
        if (self) {
          const uint32_t j = hk.inbox_slot(p ^ 1u, lt);
          if (j == ~0u) atomicOr(S.err, GG_DERR_CAP);
          else inb(S, p ^ 1u)[(size_t)lt * P.IC + j] = r;
          ri_self++;
        }
        const uint64_t m = __ballot(net);
        const uint32_t pos = nn + (uint32_t)__builtin_popcountll(m & ((1ull << ln) - 1));
        if (net) {
          const gg_cmsg& g = cur[r];
          t_[pos] = g.send_ps; s_[pos] = g.send_ps; k_[pos] = ((uint64_t)g.src << 32) | g.seq; o_[pos] = r;
          ri_net++;
        }
        nn += (uint32_t)__builtin_popcountll(m);
      }
      tsync();
      if (nn) {
        // the injection port (routePacket SEND_TILE, hop_by_hop.cc:151-159) in (time, key) order
        for (uint32_t i = ln; i < nn; i += 64) i_[i] = o_[i];
        tsync();
        if (DG(S.trs)) _q1 = __builtin_amdgcn_s_memtime();
        order_port(nn, t_, s_, k_, i_, o_, ln);
        if (DG(S.trs)) _q2 = __builtin_amdgcn_s_memtime();
        const uint64_t qi = (uint64_t)T.tile * 6 + P_INJ;
        HQueue* gq = S.nq + qi;
        HNode* gnd = S.nnd + qi * P.np.max_size;
        const bool regq = F ? P.np.qm != 0 : P.np.qm && P.np.qtype == GG_QM_HISTORY_TREE && P.np.max_size <= kQMax;
        const bool wave = !F && P.np.qm && P.np.max_size <= kQMax && !regq;
        // the port's queue: tr in HBM, trl the LDS image (one address space each:
        // a pointer merged from the two would make every queue access flat)
        HTree tr{gq, gnd, 1, P.np.analytical != 0};
        HTree trl{reinterpret_cast<HQueue*>(sl.pimg), reinterpret_cast<HNode*>(sl.pimg + sizeof(HQueue)), 1,
                  P.np.analytical != 0};
        if (wave) {
          img_in(sl.pimg, gq, gnd, P.np.max_size, ln);
          tsync();
            }
        RegQueue rq;
        if (regq) rq.load_h0(gq, gnd, P.np.max_size, 1, P.np.analytical != 0, ln);
        if (DG(S.trs)) { (void)__builtin_amdgcn_readfirstlane((int)rq.a0); _q3 = __builtin_amdgcn_s_memtime(); }
        uint64_t ps = 0, fs = 0, bs = 0;
        for (uint32_t c0 = 0; c0 < nn; c0 += 64) {
          const uint32_t cnt = min(64u, nn - c0);
          uint32_t r = 0, nf_ = 0, bits = 0;
          uint64_t sp = 0;
          if (ln < cnt) {
            r = o_[c0 + ln];
            const gg_cmsg& g = cur[r];
            sp = g.send_ps;
            bits = msg_bits(P, g.type);
            nf_ = (uint32_t)nflits(P.np, bits);
          }
          uint64_t oq = 0;
          const uint64_t x0 = DG(S.prof) && regq ? rq.A(rq.sz - 1) : 0;
          uint32_t ntail = 0;
          for (uint32_t k = 0; k < cnt; ++k) {
            const uint32_t nf = (uint32_t)__builtin_amdgcn_readlane((int)nf_, (int)k);
            uint64_t qd = 0;
            if (P.np.qm) {
              const uint64_t tc = time_to_cycles(rl64(sp, k), P.np.f);
              ntail += tc >= x0;
              if constexpr (F) qd = rq.request(tc, nf, S.err); else qd = regq ? rq.request(tc, nf, S.err) : (wave ? trl.delay_w(tc, nf, S.err, ln) : tr.delay(tc, nf, S.err));
            }
            if (ln == k) oq = qd;
            fs += nf; bs += (uint32_t)__builtin_amdgcn_readlane((int)bits, (int)k);   // updateSendCounters, uniform
          }
          ps += cnt;
          if (DG(S.prof) && ln == 0) prof_batch(S, 1, cnt, ntail);
          if (ln < cnt) {                                       // (network_model.cc:228-251)
            gg_cmsg* g = cur + r;
            g->arrival_ps = sp + lat_to_ps(0, P.np.f) + lat_to_ps(oq, P.np.f);
            g->zero_load_ps = 0;
            g->hop = T.tile;
          }
        }
        if (DG(S.trs)) _q4 = __builtin_amdgcn_s_memtime();
        if (regq) rq.store(gq, gnd);
        if (wave) { tsync(); img_out(gq, gnd, sl.pimg, P.np.max_size, ln); }
        if (ln == 0) {
          cadd(S.ctr, T.tile, GG_NC_PACKETS_SENT, ps); cadd(S.ctr, T.tile, GG_NC_FLITS_SENT, fs);
          cadd(S.ctr, T.tile, GG_NC_BITS_SENT, bs);
        }
        tsync();
        // onto the X (or Y) segment the packet enters
        for (uint32_t i = ln; i < nn; i += 64) {
          const uint32_t r = o_[i];
          bool is_x;
          const uint32_t d = cur[r].dst;
          const uint32_t sg = xy_stage_seg(P, S, T.tile, d, is_x);
          const uint32_t j = hk.seg_slot(is_x, sg);
          if (j == ~0u) { atomicOr(S.err, GG_DERR_CAP); continue; }
          (is_x ? S.xl : S.yl)[(size_t)sg * P.seg_cap + j] = (uint64_t)r | ((uint64_t)d << 32);
        }
      }
    }
    };
    if (np_ <= SL::kIn) pub_batch(std::true_type{}); else pub_batch(std::false_type{});
  }

  PROF_AT(_p4);
  // ---- 4. write back
  if (T.rq_lds) {
    CReq* g = S.rq + (size_t)lt * P.QC;
    for (uint32_t i = ln; i < T.nrq; i += 64) g[i] = sl.rq[i];
  }
  if (T.dq_lds) img_out(S.dq + lt, S.dnd + (size_t)lt * P.max_list, sl.dimg, P.max_list, ln);
  T.eclose();
  T.flush();
  T.flush_err();
  // NoC counters of the tile's own SELF port and receiver
  {
    if (na) {
      const int ci = ln == 0 ? GG_NC_ROUTER_CONTENTION_CYCLES : ln == 1 ? GG_NC_ROUTER_PACKETS
                   : ln == 2 ? GG_NC_BUFFER_WRITES : ln == 3 ? GG_NC_SWITCH_ALLOC : ln == 4 ? GG_NC_CROSSBAR
                   : ln == 5 ? GG_NC_LINK_TRAVERSALS : ln == 6 ? GG_NC_BUFFER_READS : ln == 8 ? GG_NC_PACKETS_RECEIVED
                   : ln == 9 ? GG_NC_FLITS_RECEIVED : ln == 10 ? GG_NC_BITS_RECEIVED : ln == 11 ? GG_NC_TOTAL_LATENCY_PS
                   : ln == 12 ? GG_NC_TOTAL_CONTENTION_PS : -1;
      if (ci >= 0 && ncd) cadd(S.ctr, T.tile, (uint32_t)ci, ncd);
    }
  }
  {
    const uint32_t a = wave_sum((uint32_t)ri_net), b = wave_sum((uint32_t)ri_self), c = wave_sum((uint32_t)ri_bnd);
    if (ln == 0) hk.step_counts(k, a, b, c, np_);
  }
  if (DG(S.prof) && ln == 0) {
    const uint64_t e = __builtin_amdgcn_s_memtime();
    atomicAdd(&DG(S.prof)[0], (unsigned long long)(_p1 - _p0)); atomicAdd(&DG(S.prof)[1], (unsigned long long)(_p2 - _p1));
    atomicAdd(&DG(S.prof)[2], (unsigned long long)(_p3 - _p2)); atomicAdd(&DG(S.prof)[3], (unsigned long long)(_p4 - _p3));
    atomicAdd(&DG(S.prof)[4], (unsigned long long)(e - _p4));
    atomicMax(&DG(S.prof)[1024 + (L & 65535)], (unsigned long long)(e - _p0));
    atomicMax(&DG(S.prof)[1024 + 3 * 65536 + (L & 65535)], (unsigned long long)(na + T.nsent));
    {
      // the slowest tile's shape: (total << 24) | payload, max per launch
      const uint64_t tot = (e - _p0) << 24;
      auto c8 = [](uint64_t v) { return v > 255 ? 255ull : v; };
      auto c24 = [](uint64_t v) { v >>= 8; return v > 0xFFFFFF ? 0xFFFFFFull : v; };
      const size_t b = 1024 + 6 * 65536 + 4 * (L & 16383);
      atomicMax(&DG(S.prof)[b + 0], (unsigned long long)(tot | (c8(ni) << 16) | (c8(na) << 8) | c8(T.nsent)));
      atomicMax(&DG(S.prof)[b + 1], (unsigned long long)(tot | c24(_p1 - _p0)));
      atomicMax(&DG(S.prof)[b + 2], (unsigned long long)(tot | c24(_p2 - _p1)));
      atomicMax(&DG(S.prof)[b + 3], (unsigned long long)(tot | c24(_p3 - _p2)));
    }
  }
  if (DG(S.trs) && L < S.tr_n && ln == 0) {
    unsigned long long* r = DG(S.trs) + ((size_t)L * P.L + lt) * kTrStep;
    r[2] = _p0; r[3] = _sa; r[4] = _p1; r[5] = _p2; r[6] = _p3; r[7] = _p4; r[8] = __builtin_amdgcn_s_memtime();
    r[9] = (unsigned long long)na | ((unsigned long long)ni << 16) | ((unsigned long long)T.nsent << 32);
    r[10] = _sb; r[11] = _sc; r[12] = _sd; r[13] = _se; r[14] = _q1b; r[15] = _sf;
    r[16] = _q1; r[17] = _q2; r[18] = _q3; r[19] = _q4;
    r[20] = _hd; r[21] = _hl; r[22] = _hn;
    for (int i = 0; i < 9; ++i) r[23 + i] = T.tra[i];
  }
  // the tile's next start for the shard scheduler: finished, blocked, or clock + gap
  if (T.rec >= T.rec_end) return kNsFin;
  if (T.blocked) return kNsBlk;
  return T.clk + rec_gap(S.meta[T.rec]) * P.gap_ps;
}

// The diagnostic hooks (GG_COH_PROFILE / GG_COH_TRACE: phase cycles, step and
// walker traces) are compiled only into a diagnostics build (-DGG_COH_DIAG=1,
// tools/build_variant.sh): in the product kernels their pointers are null
// constants, so the hooks and the registers they would hold are gone.

__device__ __forceinline__ void diag_off(CS& S)
{
  if (!GG_COH_DIAG) { S.prof = nullptr; S.trs = nullptr; S.trw = nullptr; S.tre = nullptr; }
}

// Scalar-cache warm-up of a launch-state block (CP / CS, read where used
// through pointers): one load per 64-B line, all issued at
// kernel entry, so the scalar-cache misses a wave would otherwise take one by
// one along its dependent path (an L2 round trip each; PMC: ~1 300 scalar
// misses per step launch) cost one latency.  The words are folded into a
// value an empty asm consumes, so the loads are kept.
#ifndef GG_KWARM
#define GG_KWARM 1
#endif
template <class A, class B>
__device__ __forceinline__ void kwarm(const A* __restrict__ a, const B* __restrict__ b)
{
  if (!GG_KWARM) return;
  const uint32_t* wa = reinterpret_cast<const uint32_t*>(a);
  const uint32_t* wb = reinterpret_cast<const uint32_t*>(b);
  constexpr uint32_t kA = (uint32_t)((sizeof(A) + 63) / 64), kB = (uint32_t)((sizeof(B) + 63) / 64);
  uint32_t x[kA + kB];
#pragma unroll
  for (uint32_t i = 0; i < kA; ++i) x[i] = wa[16 * i];
#pragma unroll
  for (uint32_t i = 0; i < kB; ++i) x[kA + i] = wb[16 * i];
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t i = 0; i < kA + kB; ++i) acc ^= x[i];
  asm volatile("; kwarm %0" ::"s"(acc));
}

// in-kernel launch timing (timing mode 2): every workgroup stamps its start
// and end (100 MHz s_memrealtime) in its own words — plain stores, no atomic
// on a shared word (1 024 blocks contending for one had added ~8 µs to the
// step kernel) — and the host takes the first start and the last end: the
// kernel's execution span as rocprofv3's kernel trace sees it
__device__ __forceinline__ void kt_begin(const CS& S)
{
  if (S.kt && threadIdx.x == 0)
    S.kt[(size_t)S.kt_slot * S.kt_stride + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void kt_end(const CS& S)
{
  if (!S.kt) return;
  __syncthreads();
  if (threadIdx.x == 0) S.kt[(size_t)S.kt_slot * S.kt_stride + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}


// ---------------------------------------------------------------------------
// hop-by-hop: one workgroup per X (stage 0) or Y (stage 1) run of routers
// (one direction).  In a run the packets move one way, so the requests a port
// sees depend only on the ports before it; the canonical order at a port is
// (arrival time, rank) over the step's packets.
// * one wave (64 threads, the persistent small-mesh kernel): the positions
//   are served in the direction of travel, each position's whole batch in
//   (time, rank) order (sweep_positions);
// * one wave per position (k_c_walk): the positions are served concurrently
//   as a pipeline.  Wave w serves its port's pending packets in (time, rank)
//   order; a packet is safe once its time is below the horizon of the wave
//   before it: that wave's published lower bound on the time of any packet it
//   will still serve, plus the router + link delay (a packet leaves a port no
//   earlier than it arrived there, plus that delay).  Same requests, same
//   order, at every port (pipeline_positions).
// ---------------------------------------------------------------------------
constexpr uint32_t kWalkSync = 512;                  // LDS: per-wave horizon / done words, run bounds
constexpr uint32_t kMaxWalkWaves = 16;
#ifndef GG_WALK_SLEEP
#define GG_WALK_SLEEP 1                              // s_sleep units (64 cycles) between horizon polls
#endif

__device__ __forceinline__ uint64_t wave_min64(uint64_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const uint64_t u = (uint64_t)__shfl_xor((long long)v, o); v = u < v ? u : v; }
  return v;
}
__device__ __forceinline__ uint64_t lds_load_acq(const uint64_t* p)
{
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint64_t* p, uint64_t v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the pipeline's packet word: time << 12 | position << 2 | status (times
// < 2^51 are checked at staging; positions < 1024)
__device__ __forceinline__ uint64_t pipe_word(uint64_t t, uint32_t pos, uint32_t status)
{
  return (t << 12) | ((uint64_t)pos << 2) | status;
}
__device__ __forceinline__ uint32_t pipe_pos(uint64_t w) { return (uint32_t)(w >> 2) & 0x3FFu; }

struct WalkLds {
  uint64_t *Pt, *Ph, *Pk, *Pz;
  uint32_t *Pi, *Pp, *Pd, *Pf, *Pr;
  uint64_t *Qt; uint32_t *Qr, *Qs;
};

// the port of position pos serves one packet i (RouterModel + link, the
// canonical request): queue delay at the port, router + link delay; the
// packet moves to the next position (status 2: held at the shard's edge, 1:
// leaves the run, 0: continues)
template <class Q>
__device__ __forceinline__ uint64_t serve_packet(const CP& P, const CS& S, const WalkLds& W, Q&& request, uint32_t i,
                                                 uint32_t nx, const Seg& sd, uint64_t zps, uint64_t& cf)
{
  const uint64_t t = W.Pt[i];
  const uint32_t f = W.Pf[i], nf = f & 0xFFFFFFu, d = W.Pd[i];
  const uint64_t qd = request(t, nf);
  cf += nf;
  uint32_t status = 0;
  if (nx < sd.lo || nx > sd.hi) status = 2;            // next router in another shard: held
  else if (nx == d) status = 1;                        // leaves the run: next stage
  W.Pt[i] = t + zps + lat_to_ps(qd, P.np.f);
  W.Pz[i] += zps;
  W.Pf[i] = nf | (status << 24);
  return qd;
}

// RQ: the ports' queues are history trees held in registers (RegQueue;
// walk_regq) — a separate instance, so the pipeline loop carries only that
// request path (no LDS-image / list / M/G/1-only code, no spills)
__host__ __device__ inline bool walk_regq(const CP& P)
{
  return P.np.qm && P.np.qtype == GG_QM_HISTORY_TREE && P.np.max_size <= kQMax;
}

template <bool PIPE, bool RQ>
__device__ __forceinline__ void walk_body(const CP& P, const CS& S, uint32_t L, int stage, uint32_t blk)
{
  // block -> (run slot, direction): with runs interleaved by shard, block b
  // takes slot (b mod ns) + ns * (b div 2ns) in direction (b div ns) & 1, so
  // every block of shard k is k mod ns (the XCD of its tiles' blocks)
  uint32_t sg = blk;
  if (P.seg_xcd) {
    const uint32_t ns = P.seg_xcd, b = blk;
    sg = 2 * ((b % ns) + ns * (b / (2 * ns))) + ((b / ns) & 1u);
  }
  const uint32_t tid = threadIdx.x, nthr = blockDim.x, ln = tid & 63;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));   // wave-uniform: SGPR control flow
  // one round of loads: the launch's live word, the run's count and bounds,
  // and (speculatively: in bounds whatever the count) its first list words
  uint32_t* cntp = (stage == 0 ? S.nxl : S.nyl) + sg;
  const uint64_t* list = (stage == 0 ? S.xl : S.yl) + (size_t)sg * P.seg_cap;
  const uint32_t live = S.live[L & 3];
  const uint32_t n0 = *cntp;
  const Seg sd = (stage == 0 ? S.segx : S.segy)[sg >> 1];
  const uint64_t lw = tid < P.seg_cap ? list[tid] : 0ull;
  if (!live) return;                                 // launch L was no step
  const uint32_t p = (live - 1) & 1u;
  PROF_T0();
  if (n0 == 0) return;
  const uint32_t n = min(n0, P.seg_cap);
  const uint32_t dir = sg & 1u;
  const int port = stage == 0 ? (dir ? P_RIGHT : P_LEFT) : (dir ? P_UP : P_DOWN);
  auto tile_at = [&](uint32_t pos) -> uint32_t { return stage == 0 ? sd.line * P.mw + pos : pos * P.mw + sd.line; };
  auto pos_of = [&](uint32_t tile) -> uint32_t { return stage == 0 ? tile % P.mw : tile / P.mw; };
  gg_cmsg* cur = pool(S, p);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t npos = sd.hi - sd.lo + 1;
  const bool qm = RQ || P.np.qm != 0;
  constexpr bool regq = RQ;
  const bool sweep = !PIPE || n > 128 || P.walk_wide;     // more than 128 packets (or the A/B knob): wave 0 sweeps
  // the pipeline with register queues: each wave loads its port's history
  // tree straight from HBM into registers now, beside the packet staging
  // (no LDS image copy in or out; written back only if the port served)
  const bool direct = PIPE && regq && !sweep;
  // (issued right after the lane's packet record loads below, read after
  // them: the queue's round trip and the records' overlap)
  RegQueue rq;
  RegQueue::Raw rqr;
  const bool rq_direct = direct && wv < npos;
  const uint64_t rq_qi = rq_direct ? (uint64_t)tile_at(dir ? sd.lo + wv : sd.hi - wv) * 6 + port : 0ull;
  uint8_t* qimg = smem;
  uint64_t* lc = reinterpret_cast<uint64_t*>(smem + (size_t)npos * P.qimg);     // [npos][kNetCtr]
  uint64_t* wlow = lc + (size_t)npos * kNetCtr;                                  // [kMaxWalkWaves] horizons (kInf: done)
  uint32_t* rlohi = reinterpret_cast<uint32_t*>(wlow + kMaxWalkWaves);           // lo, ~hi of the visited positions
  uint8_t* pk = reinterpret_cast<uint8_t*>(wlow) + kWalkSync;
  if (n > P.walk_pk) { if (tid == 0) { atomicOr(S.err, GG_DERR_CAP); *cntp = 0; } return; }
  WalkLds W;
  W.Pt = reinterpret_cast<uint64_t*>(pk);
  W.Ph = W.Pt + P.walk_pk; W.Pk = W.Ph + P.walk_pk; W.Pz = W.Pk + P.walk_pk;
  W.Pi = reinterpret_cast<uint32_t*>(W.Pz + P.walk_pk);
  W.Pp = W.Pi + P.walk_pk; W.Pd = W.Pp + P.walk_pk; W.Pf = W.Pd + P.walk_pk;   // pos, exit pos, flits | status << 24
  W.Pr = W.Pf + P.walk_pk;                                       // rank in (send time, sender, seq) order
  W.Qt = reinterpret_cast<uint64_t*>(W.Pr + P.walk_pk);          // batch scratch of the one-wave sweep
  W.Qr = reinterpret_cast<uint32_t*>(W.Qt + P.walk_pk); W.Qs = W.Qr + P.walk_pk;
  // The hand-off of lane i == tid's packet (the common case) is prepared
  // here, beside the record loads: the destination comes with the list
  // entry, so the receiver's local slot (the run ends at the destination) or
  // the Y run the packet turns into is looked up in the same round as the
  // records; where the packet leaves the run is known before the walk (at
  // the destination's position, or held at the shard's edge when that lies
  // beyond the run), so its slot in the next list is reserved right after
  // staging and the walk hides that atomic's round trip; a held packet's
  // other record fields are read now for its boundary copy.  The hand-off
  // then only stores.
  uint32_t pdst = 0, pf = 0;
  bool pheld = false;
  uint64_t haddr = 0;
  uint32_t hreq = 0, htype = 0, hlink = 0, hsrx = 0;
  // lane tid's packet first, with no loop around it (so the waits for its
  // record are counted, not drained): record fields and lookups, then the
  // port queue's loads, then the record into LDS
  // (unconditional loads — a lane without a packet reads record 0 and
  // tile 0 — so no branch merges their registers before the queue's issue)
  const bool has_p = tid < n;
  const uint32_t orec = has_p ? (uint32_t)lw : 0u;
  pdst = has_p ? (uint32_t)(lw >> 32) : 0u;
  const gg_cmsg& om = cur[orec];
  const uint64_t ot = om.arrival_ps, os = om.send_ps, oz = om.zero_load_ps;
  const uint32_t osrc = om.src, oseq = om.seq, ohop = om.hop, otype = om.type;
  haddr = om.addr; hreq = om.requester; hlink = om.link; hsrx = om.single_rx;
  {
    const uint32_t z = pos_of(pdst);
    pheld = has_p && (z < sd.lo || z > sd.hi);
    const uint32_t hx = tile_at(z);
    pf = hx == pdst ? (uint32_t)S.ltile[pdst] : S.tseg[(size_t)hx * 2 + 1];
  }
  if (rq_direct) rqr = RegQueue::issue(S.nq + rq_qi, S.nnd + rq_qi * P.np.max_size, P.np.max_size, ln);
  if (tid < n) {
    const uint32_t i = tid;
    htype = otype;
    W.Pt[i] = ot; W.Ph[i] = os; W.Pk[i] = ((uint64_t)osrc << 32) | oseq; W.Pz[i] = oz;
    W.Pi[i] = orec; W.Pp[i] = pos_of(ohop); W.Pd[i] = pos_of(pdst);
    if (ot >> 51) atomicOr(S.err, GG_DERR_CAP);                  // batch keys are time << 12 | rank
    W.Pf[i] = (uint32_t)nflits(P.np, msg_bits(P, otype));
  }
  for (uint32_t i = tid + nthr; i < n; i += nthr) {               // more packets than threads
    const uint64_t le = list[i];
    const uint32_t r = (uint32_t)le;
    const gg_cmsg& m = cur[r];
    W.Pt[i] = m.arrival_ps; W.Ph[i] = m.send_ps; W.Pk[i] = ((uint64_t)m.src << 32) | m.seq; W.Pz[i] = m.zero_load_ps;
    W.Pi[i] = r; W.Pp[i] = pos_of(m.hop); W.Pd[i] = pos_of(m.dst);
    if (m.arrival_ps >> 51) atomicOr(S.err, GG_DERR_CAP);
    W.Pf[i] = (uint32_t)nflits(P.np, msg_bits(P, m.type));
  }
  if (rq_direct) rq.finish(rqr, S.nq + rq_qi, S.nnd + rq_qi * P.np.max_size, 1, P.np.analytical != 0, ln);
  // lane tid's slot in the list its packet moves to (a held record, a SELF
  // list, a Y run): reserved when the wave's walk is over, so the atomic's
  // round trip overlaps the other waves' (the raw result is checked at the
  // hand-off)
  uint32_t jres = ~0u, s2res = 0;
  bool pself = false;
  if (!sweep)                     // the pipeline's moving state: one word per packet (W.Qt, unused by it)
    for (uint32_t i = tid; i < n; i += nthr) W.Qt[i] = pipe_word(W.Pt[i], W.Pp[i], 0u);
  for (uint32_t i = tid; i < npos * kNetCtr; i += nthr) lc[i] = 0;
  for (uint32_t i = tid; i < kMaxWalkWaves; i += nthr) wlow[i] = 0;
  if (tid == 0) { rlohi[0] = ~0u; rlohi[1] = ~0u; rlohi[2] = 0; }
  __syncthreads();
  // canonical ranks (by send time, sender, seq); the positions the packets can visit
  if (!PIPE) {
    for (uint32_t i = tid; i < n; i += nthr) {
      const uint64_t hi_ = W.Ph[i], ki = W.Pk[i];
      uint32_t r = 0;
      for (uint32_t j = 0; j < n; ++j) { const uint64_t hj = W.Ph[j]; r += hj < hi_ || (hj == hi_ && W.Pk[j] < ki); }
      W.Pr[i] = r;
    }
  } else {
    // a wave per packet: its lanes compare against 64 packets at a time
    const uint32_t nw = nthr >> 6;
    for (uint32_t i = wv; i < n; i += nw) {
      const uint64_t hi_ = W.Ph[i], ki = W.Pk[i];
      uint32_t r = 0;
      for (uint32_t b0 = 0; b0 < n; b0 += 64) {
        const uint32_t j = b0 + ln;
        bool lt = false;
        if (j < n) { const uint64_t hj = W.Ph[j]; lt = hj < hi_ || (hj == hi_ && W.Pk[j] < ki); }
        r += (uint32_t)__builtin_popcountll(__ballot(lt));
      }
      if (ln == 0) W.Pr[i] = r;
    }
  }
  uint32_t lo = ~0u, hi = 0;
  for (uint32_t i = tid; i < n; i += nthr) {
    const uint32_t a = W.Pp[i], z = W.Pd[i];
    const uint32_t zz = dir ? min(z - 1, sd.hi) : max(z + 1, sd.lo);
    lo = min(lo, min(a, zz)); hi = max(hi, max(a, zz));
  }
  lo = wave_min(lo);
  hi = (uint32_t)(~wave_min(~hi));
  if (ln == 0 && lo != ~0u) { atomicMin(&rlohi[0], lo); atomicMin(&rlohi[1], ~hi); }
  __syncthreads();
  lo = rlohi[0]; hi = ~rlohi[1];
  auto qi_of = [&](uint32_t i) { return (uint64_t)tile_at(lo + i) * 6 + port; };
  if (qm && lo <= hi && !direct)
    imgs_copy<true, decltype(qi_of), 4>(qimg + (size_t)(lo - sd.lo) * P.qimg, P.qimg, hi - lo + 1, qi_of, S.nq, S.nnd,
                                        P.np.max_size, tid, nthr);
  __syncthreads();
  PROF_AT(_w1);
  const bool wave_q = P.np.max_size <= kQMax;
  const uint64_t zps = rfl64(lat_to_ps((uint64_t)P.np.router_delay + P.np.link_delay, P.np.f));   // scalar
  uint32_t nev = 0;
  // the port of one position, its queue in registers (history tree) or the LDS image
  auto port_queue = [&](uint32_t pos, RegQueue& rq, HTree& tr) {
    uint8_t* im = qimg + (size_t)(pos - sd.lo) * P.qimg;
    tr = HTree{reinterpret_cast<HQueue*>(im), reinterpret_cast<HNode*>(im + sizeof(HQueue)), 1, P.np.analytical != 0};
    if (regq) rq.load(tr.q, tr.nd, 1, P.np.analytical != 0, ln);
  };
  auto add_ctr = [&](uint32_t pos, uint64_t cq, uint64_t m, uint64_t cf) {
    // port_hop's counters: contention, router packets, buffer w+r, switch, crossbar, link
    uint64_t* l = lc + (size_t)(pos - sd.lo) * kNetCtr;
    l[0] += qm ? cq : 0; l[1] += qm ? m : 0; l[2] += cf; l[3] += m; l[4] += cf; l[5] += cf;
  };
  if (sweep && wv == 0) {
    // ---- one wave: position sweep, each position's batch in (time, rank) order
    uint64_t* K = W.Qt; uint32_t* B = W.Qr; uint32_t* O = W.Qs;
    for (uint32_t s_ = 0; lo <= hi && s_ <= hi - lo; ++s_) {
      const uint32_t pos = dir ? lo + s_ : hi - s_;
      uint32_t m = 0;
      for (uint32_t b0 = 0; b0 < n; b0 += 64) {
        const uint32_t i = b0 + ln;
        const bool at = i < n && W.Pp[i] == pos && (W.Pf[i] >> 24) == 0;
        const uint64_t bm = __ballot(at);
        if (at) {
          const uint32_t k = m + (uint32_t)__builtin_popcountll(bm & ((1ull << ln) - 1));
          B[k] = i; K[k] = (W.Pt[i] << 12) | W.Pr[i];
        }
        m += (uint32_t)__builtin_popcountll(bm);
      }
      if (m == 0) continue;
      wave_sync();
      for (uint32_t k = ln; k < m; k += 64) {
        const uint64_t kk = K[k];
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) r += K[j] < kk;
        O[r] = B[k];
      }
      wave_sync();
      RegQueue rq; HTree tr;
      port_queue(pos, rq, tr);
      auto request = [&](uint64_t t, uint32_t nf) -> uint64_t {
        if (!qm) return 0;
        const uint64_t tc = time_to_cycles(t, P.np.f);
        return regq ? rq.request<false>(tc, nf, S.err) : (wave_q ? tr.delay_w(tc, nf, S.err, ln) : tr.delay(tc, nf, S.err));
      };
      const uint32_t nx = dir ? pos + 1 : pos - 1;
      uint64_t cq = 0, cf = 0;
      for (uint32_t k = 0; k < m; ++k) {
        const uint32_t i = O[k];
        cq += serve_packet(P, S, W, request, i, nx, sd, zps, cf);
        if (ln == 0) W.Pp[i] = nx;
        wave_sync();
      }
      nev += m;
      if (regq) rq.store(tr.q, tr.nd);
      if (ln == 0) add_ctr(pos, cq, m, cf);
      wave_sync();
    }
  } else if (!sweep && wv < npos) {
    // ---- one wave per position (blockDim.x = 64 x positions): the pipeline
    // (n <= 128: lane l watches packets l and l + 64 if their route crosses
    // this port; the wide case took the sweep above)
    const uint32_t pos = dir ? sd.lo + wv : sd.hi - wv;
    const uint32_t nx = dir ? pos + 1 : pos - 1;
    constexpr uint64_t kInf = ~0ull;
    const bool visited = lo <= hi && pos >= lo && pos <= hi;
    HTree tr;
    if (visited && !direct) port_queue(pos, rq, tr);
    const uint32_t status_nx = (nx < sd.lo || nx > sd.hi) ? 2u : 0u;   // next router in another shard: held
    uint64_t cq = 0, cf = 0, m = 0;
    uint32_t spin = 0, polls = 0;
    const bool tev = DG(S.tre) && L >= kTrEv0 && L < kTrEv0 + S.tre_n;
    unsigned long long* tre = tev ? DG(S.tre) + (((size_t)(L - kTrEv0) * 2 + stage) * S.tr_wb + blk) * (kTrEvMax * 4 + 4) : nullptr;
    auto crosses = [&](uint32_t i) {
      if (i >= n) return false;
      const uint32_t a = W.Pp[i], z = W.Pd[i];
      return dir ? (a <= pos && pos < z) : (a >= pos && pos > z);
    };
    // per lane: its packets' rank, flits and exit position (fixed) in registers
    bool c0 = visited && crosses(ln), c1 = visited && crosses(ln + 64);
    const uint32_t r0 = c0 ? W.Pr[ln] : 0u, r1 = c1 ? W.Pr[ln + 64] : 0u;
    const uint32_t fd0 = c0 ? (W.Pf[ln] & 0xFFFFFFu) | (W.Pd[ln] << 24) : 0u;   // flits (< 2^24) | exit pos << 24
    const uint32_t fd1 = c1 ? (W.Pf[ln + 64] & 0xFFFFFFu) | (W.Pd[ln + 64] << 24) : 0u;
    uint64_t* wup = wv > 0 ? &wlow[wv - 1] : nullptr;
    // one loop exit, a readfirstlane'd flag: the loop is wave-uniform, so its
    // carried values stay scalar (no exec-masked loop, no VGPR phis)
    uint32_t go = visited ? 1u : 0u;
    uint64_t last_ul = 0;
    bool waiting = false;
    while (__builtin_amdgcn_readfirstlane((int)go)) {
      // the horizon, in canonical keys (time << 12 | rank): the wave before
      // publishes a lower bound on the key of every packet it will still
      // serve (kInf once it has served its last one); such a packet reaches
      // this port with a key at least that bound + zps << 12, so every
      // pending packet with a key <= bound here is safe (keys are unique).
      // A packet forwarded upstream with no queue delay is therefore safe at
      // once, without waiting for the upstream port to move on.
      uint64_t bound = kInf;
      if (wup) {
        const uint64_t ul = rq.rd64(lds_load_acq(wup));          // uniform (an atomic load is taken as divergent)
        // a waiting wave re-evaluates only when the upstream word moved: every
        // packet the wave before forwards comes with a new (larger) word, so
        // an unchanged word means nothing new (the cheap poll keeps the
        // waiting waves off the serving waves' issue slots)
        if (waiting && ul == last_ul) {
          if (++spin > (1u << 22)) { if (ln == 0) atomicOr(S.err, GG_DERR_STATE); go = 0; continue; }
          __builtin_amdgcn_s_sleep(GG_WALK_SLEEP);
          continue;
        }
        last_ul = ul;
        bound = ul == kInf ? kInf : ul + (zps << 12);
      }
      waiting = false;
      const bool up_fin = bound == kInf;
      // the least pending packet at this position, by (time, rank): each lane
      // its least (the packet words, read after the acquire of the horizon
      // word: every packet forwarded before that word was written is seen),
      // then a scalar pass over the lanes holding one
      const uint64_t w0 = c0 ? W.Qt[ln] : ~0ull;
      const uint64_t w1 = c1 ? W.Qt[ln + 64] : ~0ull;
      uint64_t mk = kInf;
      uint32_t mi = 0, mfd = 0;
      if (pipe_pos(w0) == pos) { mk = (w0 & ~0xFFFull) | r0; mi = ln; mfd = fd0; }
      if (pipe_pos(w1) == pos) {
        const uint64_t k = (w1 & ~0xFFFull) | r1;
        if (k < mk) { mk = k; mi = ln + 64; mfd = fd1; }
      }
      uint64_t wk = kInf;
      uint32_t wl = 0;
      for (uint64_t bm = __ballot(mk != kInf); bm; bm &= bm - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(bm);
        const uint64_t k = rl64(mk, l);
        if (k < wk) { wk = k; wl = l; }
      }
      if (wk == kInf && up_fin) { go = 0; continue; }                   // nothing pending, nothing to come
      if (wk > bound) {
        // wait for upstream progress; publish the least key this port can still serve
        if (ln == 0) lds_store_rel(&wlow[wv], wk < bound ? wk : bound);
        if (++spin > (1u << 22)) { if (ln == 0) atomicOr(S.err, GG_DERR_STATE); go = 0; continue; }
        ++polls;
        waiting = true;
        __builtin_amdgcn_s_sleep(GG_WALK_SLEEP);
        continue;
      }
      const uint64_t T = wk >> 12;
      const uint64_t ev0 = tev ? __builtin_amdgcn_s_memtime() : 0;
      // serve it: the router + link (serve_packet's arithmetic); the packet
      // moves downstream as soon as its queue delay is known, the port's
      // queue is updated after that (request_pub)
      const uint32_t i = (uint32_t)__builtin_amdgcn_readlane((int)mi, (int)wl);
      const uint32_t fd = (uint32_t)__builtin_amdgcn_readlane((int)mfd, (int)wl);
      const uint32_t nf = fd & 0xFFFFFFu;
      const uint32_t status = status_nx ? status_nx : (nx == (fd >> 24) ? 1u : 0u);   // 1: leaves the run
      uint64_t evp = 0;
      auto pub = [&](uint64_t qd) {
        if (tev) evp = __builtin_amdgcn_s_memtime();
        if (ln == 0) {
          // the packet word (time, next position, status; the zero-load part,
          // + zps per port, is added at the hand-off), then the horizon
          // (release: the word is visible first)
          W.Qt[i] = pipe_word(T + zps + lat_to_ps(qd, P.np.f), nx, status);
          lds_store_rel(&wlow[wv], wk + 1);                   // every later key served here is > wk
        }
      };
      uint64_t qd = 0;
      if (!qm) pub(0ull);
      else {
        const uint64_t tc = rfl64(time_to_cycles(T, P.np.f));
        if (regq) qd = rq.request_pub(tc, nf, pub);
        else { qd = wave_q ? tr.delay_w(tc, nf, S.err, ln) : tr.delay(tc, nf, S.err); pub(qd); }
      }
      const uint64_t ev1 = tev ? __builtin_amdgcn_s_memtime() : 0;
      cq += qd; cf += nf; ++m;
      if (ln == (i & 63)) { if (i < 64) c0 = false; else c1 = false; }   // served here: no longer a candidate
      if (tev && ln == 0) {
        const uint32_t k = atomicAdd(reinterpret_cast<unsigned int*>(&rlohi[2]), 1u);
        if (k < kTrEvMax) {
          unsigned long long* e = tre + 4 + 4 * k;
          e[0] = ev0; e[1] = evp; e[2] = ev1;
          e[3] = (unsigned long long)i | ((unsigned long long)pos << 16) | ((unsigned long long)wv << 24) |
                 ((unsigned long long)polls << 32);
        }
      }
      wave_sync();
    }
    if (ln == 0) lds_store_rel(&wlow[wv], kInf);
    if (regq && visited && direct && m) {
      const uint64_t qi = (uint64_t)tile_at(pos) * 6 + port;
      rq.errp = S.err; rq.store(S.nq + qi, S.nnd + qi * P.np.max_size);
    } else if (regq && visited && !direct) {
      rq.errp = S.err; rq.store(tr.q, tr.nd);
    }
    if (ln == 0 && visited) add_ctr(pos, cq, m, cf);
    nev = (uint32_t)m;
  }
  if (tid < n) {
    const uint32_t hx = tile_at(pos_of(pdst));
    pself = !pheld && hx == pdst;
    if (pheld) jres = atomicAdd(S.bnd_cnt, 1u);
    else if (pself) jres = atomicAdd(narv_at(S, p ^ 1u, pf), 1u);
    else { s2res = pf * 2 + (pdst / P.mw > hx / P.mw ? 1u : 0u); jres = atomicAdd(&S.nyl[s2res], 1u); }
  }
  __syncthreads();
  PROF_AT(_w2);
  // hand-off
  uint32_t nb = 0;
  for (uint32_t i = tid; i < n; i += nthr) {
    const uint32_t r = W.Pi[i];
    uint32_t stt = W.Pf[i] >> 24, p1 = W.Pp[i];
    uint64_t ta = W.Pt[i], z = W.Pz[i];
    gg_cmsg* m = cur + r;
    if (!sweep) {                                              // the pipeline's word; it adds zps per port here
      const uint64_t w = W.Qt[i];
      const uint32_t p0 = p1;
      ta = w >> 12; p1 = pipe_pos(w); stt = (uint32_t)w & 3u;
      z += (uint64_t)(dir ? p1 - p0 : p0 - p1) * zps;
    }
    const uint32_t h = tile_at(p1);
    m->arrival_ps = ta; m->zero_load_ps = z; m->hop = h;
    const bool own = i == tid;                                 // this lane's packet: its slot is reserved
    if (stt == 2) {                                            // held for the quantum boundary
      if (own && !pheld) { atomicOr(S.err, GG_DERR_STATE); continue; }
      const uint32_t j = own ? jres : atomicAdd(S.bnd_cnt, 1u);
      if (j >= P.msg_cap) { atomicOr(S.err, GG_DERR_CAP); continue; }
      gg_cmsg g;
      if (own) {
        const uint64_t kk = W.Pk[i];
        g.addr = haddr; g.send_ps = W.Ph[i]; g.src = (uint32_t)(kk >> 32); g.dst = pdst; g.requester = hreq;
        g.seq = (uint32_t)kk; g.type = htype; g.link = hlink; g.single_rx = hsrx;
      } else {
        g = *m;
      }
      g.arrival_ps = ta; g.zero_load_ps = z; g.hop = h;
      S.bnd[j] = g;
      ++nb;
      continue;
    }
    const uint32_t dst = own ? pdst : m->dst;
    if (own && (pheld || pself != (h == dst))) { atomicOr(S.err, GG_DERR_STATE); continue; }   // left where staging said
    if (h == dst) {                                            // the SELF port of the destination, next step
      const int32_t ld = own ? (int32_t)pf : S.ltile[dst];
      const uint32_t j = own ? jres : atomicAdd(narv_at(S, p ^ 1u, ld), 1u);
      if (j >= P.IC) { atomicOr(S.err, GG_DERR_CAP); continue; }
      arv(S, p ^ 1u)[(size_t)ld * P.IC + j] = r;
    } else {                                                   // X done: the Y segment of the destination column
      bool is_x;
      const uint32_t s2 = own ? s2res : xy_stage_seg(P, S, h, dst, is_x);
      const uint32_t j = own ? jres : atomicAdd(&S.nyl[s2], 1u);
      if (j >= P.seg_cap) { atomicOr(S.err, GG_DERR_CAP); continue; }
      S.yl[(size_t)s2 * P.seg_cap + j] = (uint64_t)r | ((uint64_t)dst << 32);
    }
  }
  nb = wave_sum(nb);
  if (ln == 0 && nb) atomicAdd((unsigned long long*)&S.ri[GG_RI_BOUNDARY_MSGS], (unsigned long long)nb);
  if (qm && lo <= hi && !direct)
    imgs_copy<false, decltype(qi_of), 4>(qimg + (size_t)(lo - sd.lo) * P.qimg, P.qimg, hi - lo + 1, qi_of, S.nq, S.nnd,
                                         P.np.max_size, tid, nthr);
  for (uint32_t i = tid; i < npos * 6u; i += nthr) {
    const uint32_t q = i / 6, f = i % 6;
    const uint64_t* l = lc + (size_t)q * kNetCtr;
    const uint32_t tl = tile_at(sd.lo + q);
    switch (f) {
    case 0: cadd(S.ctr, tl, GG_NC_ROUTER_CONTENTION_CYCLES, l[0]); break;
    case 1: cadd(S.ctr, tl, GG_NC_ROUTER_PACKETS, l[1]); break;
    case 2: cadd(S.ctr, tl, GG_NC_BUFFER_WRITES, l[2]); cadd(S.ctr, tl, GG_NC_BUFFER_READS, l[2]); break;
    case 3: cadd(S.ctr, tl, GG_NC_SWITCH_ALLOC, l[3]); break;
    case 4: cadd(S.ctr, tl, GG_NC_CROSSBAR, l[4]); break;
    default: cadd(S.ctr, tl, GG_NC_LINK_TRAVERSALS, l[5]); break;
    }
  }
  if (tid == 0) *cntp = 0;
  if (DG(S.tre) && L >= kTrEv0 && L < kTrEv0 + S.tre_n && tid == 0) {
    unsigned long long* e = DG(S.tre) + (((size_t)(L - kTrEv0) * 2 + stage) * S.tr_wb + blk) * (kTrEvMax * 4 + 4);
    e[0] = rlohi[2]; e[1] = _w1; e[2] = _w2; e[3] = n | ((unsigned long long)npos << 32);
  }
  if (DG(S.trs) && L < S.tr_n) {
    nev = wave_sum(ln == 0 ? nev : 0u);
    __shared__ uint32_t tr_ev;
    if (tid == 0) tr_ev = 0;
    __syncthreads();
    if (ln == 0) atomicAdd(&tr_ev, nev);
    __syncthreads();
    if (tid == 0) {
      unsigned long long* r = DG(S.trw) + (((size_t)L * 2 + stage) * S.tr_wb + blk) * 8;
      r[1] = __builtin_amdgcn_s_memrealtime();
      r[2] = _p0; r[3] = _w1; r[4] = _w2; r[5] = __builtin_amdgcn_s_memtime();
      r[6] = (unsigned long long)n | ((unsigned long long)npos << 32); r[7] = tr_ev;
    }
  }
  if (DG(S.prof)) {
    nev = wave_sum(ln == 0 ? nev : 0u);
    if (ln == 0) {
      const uint64_t e = __builtin_amdgcn_s_memtime();
      atomicAdd(&DG(S.prof)[19], (unsigned long long)nev);
      if (wv == 0) {
        atomicAdd(&DG(S.prof)[16], (unsigned long long)(_w1 - _p0)); atomicAdd(&DG(S.prof)[17], (unsigned long long)(_w2 - _w1));
        atomicAdd(&DG(S.prof)[18], (unsigned long long)(e - _w2));
        atomicAdd(&DG(S.prof)[22], 1ull);
        atomicMax(&DG(S.prof)[1024 + 65536 + 2 * (L & 65535) + stage], (unsigned long long)(e - _p0));
      }
      atomicMax(&DG(S.prof)[24 + stage], (unsigned long long)nev);
    }
  }
}

// A barrier of every workgroup of the launch (one wave each): release of the
// wave's stores, an arrival count, a relaxed poll, an acquire
// (MI355X_MICROARCH.md, inter-workgroup visibility).  The poll is bounded: a
// barrier that never completes flags GG_DERR_STATE instead of hanging.
__device__ __forceinline__ void grid_sync(const CS& S, uint32_t& gen)
{
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    ++gen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(S.gbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = gen * gridDim.x;
    for (uint32_t spin = 0; __hip_atomic_load(S.gbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
      if (spin > (1u << 24)) { atomicOr(S.err, GG_DERR_STATE); break; }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// The last barrier of a persistent step, with the run's stop vote: each block
// reads the run-over and error flags after its own step (its writes are
// visible to it) and ORs them into a vote word before arriving; after the
// barrier every block reads the same OR, so all leave the loop at the same
// step without a second barrier.  Three vote words rotate by generation:
// block 0 clears the next one before arriving (no block votes in it before
// passing this barrier), and the one it clears was last read before the
// previous barrier.
__device__ __forceinline__ uint32_t grid_sync_stop(const CS& S, uint32_t& gen)
{
  __shared__ uint32_t stop;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    ++gen;
    uint32_t* vw = S.gbar + 1;
    const uint64_t done = __hip_atomic_load(&S.qs[QS_DONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t e = __hip_atomic_load(S.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done || e) __hip_atomic_fetch_or(&vw[gen % 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) __hip_atomic_store(&vw[(gen + 1) % 3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(S.gbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = gen * gridDim.x;
    for (uint32_t spin = 0; __hip_atomic_load(S.gbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
      if (spin > (1u << 24)) { atomicOr(S.err, GG_DERR_STATE); break; }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    stop = __hip_atomic_load(&vw[gen % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return stop;
}

// Small meshes (P.L <= kPersistTiles): the device-driven loop of
// gg_coherent_run in ONE launch — launch indices [L0, L1) of step + X walk +
// Y walk, separated by grid barriers instead of kernel boundaries.  Every
// workgroup holds one owned tile (its step) and walks runs b, b + grid, ...
// LC (closed-form networks): the workgroup's tile keeps its L1-D / L2 state in
// LDS for the whole launch, loaded at the start, written back at the end.
template <bool LC>
__device__ __forceinline__ void cache_state_copy(const CP& P, const CS& S, uint32_t lt, uint8_t* clds, bool in)
{
  const size_t n1 = (size_t)P.s1 * P.a1, n2 = (size_t)P.s2 * P.a2;
  uint64_t* t1 = reinterpret_cast<uint64_t*>(clds);
  uint64_t* t2 = t1 + n1;
  uint8_t* m1 = reinterpret_cast<uint8_t*>(t2 + n2);
  uint8_t* m2 = m1 + n1;
  uint8_t* r1 = m2 + n2;
  uint8_t* r2 = r1 + P.s1;
  uint64_t* g1 = S.l1_tag + lt * n1; uint64_t* g2 = S.l2_tag + lt * n2;
  uint8_t* gm1 = S.l1_meta + lt * n1; uint8_t* gm2 = S.l2_meta + lt * n2;
  uint8_t* gr1 = S.l1_rr + (size_t)lt * P.s1; uint8_t* gr2 = S.l2_rr + (size_t)lt * P.s2;
  for (size_t i = threadIdx.x; i < n1; i += 64) { if (in) { t1[i] = g1[i]; m1[i] = gm1[i]; } else { g1[i] = t1[i]; gm1[i] = m1[i]; } }
  for (size_t i = threadIdx.x; i < n2; i += 64) { if (in) { t2[i] = g2[i]; m2[i] = gm2[i]; } else { g2[i] = t2[i]; gm2[i] = m2[i]; } }
  for (size_t i = threadIdx.x; i < P.s1; i += 64) { if (in) r1[i] = gr1[i]; else gr1[i] = r1[i]; }
  for (size_t i = threadIdx.x; i < P.s2; i += 64) { if (in) r2[i] = gr2[i]; else gr2[i] = r2[i]; }
  __syncthreads();
}

// Deliver a record of the quantum boundary: a message into the inbox of the
// quantum's first step (records in pool 1), a held packet back into the walk
// of that step (records in pool 0): the X / Y segment at its router, or the
// destination's SELF list of step 1.  `resumed` counts the held packets.
__device__ __forceinline__ void import_one(const CP& P, const CS& S, const gg_cmsg& m, uint32_t* resumed)
{
  const uint32_t at = m.hop == GG_HOP_NONE ? m.dst : m.hop;
  if (at >= P.T || m.dst >= P.T || S.ltile[at] < 0) { atomicOr(S.err, GG_DERR_STATE); return; }
  if (m.hop == GG_HOP_NONE) {
    const uint32_t r = atomicAdd(&S.npool[1], 1u);
    if (r >= P.msg_cap) { atomicOr(S.err, GG_DERR_CAP); return; }
    S.pool1[r] = m;
    const int32_t ld = S.ltile[m.dst];
    const uint32_t j = atomicAdd(ninb_at(S, 0, ld), 1u);
    if (j >= P.IC) { atomicOr(S.err, GG_DERR_CAP); return; }
    S.inb0[(size_t)ld * P.IC + j] = r;
    return;
  }
  const uint32_t r = atomicAdd(&S.npool[0], 1u);
  if (r >= P.msg_cap) { atomicOr(S.err, GG_DERR_CAP); return; }
  S.pool0[r] = m;
  atomicAdd(resumed, 1u);
  if (m.hop == m.dst) {
    const int32_t ld = S.ltile[m.dst];
    const uint32_t j = atomicAdd(narv_at(S, 1, ld), 1u);
    if (j >= P.IC) { atomicOr(S.err, GG_DERR_CAP); return; }
    S.arv1[(size_t)ld * P.IC + j] = r;
    return;
  }
  bool is_x;
  const uint32_t sg = xy_stage_seg(P, S, m.hop, m.dst, is_x);
  uint32_t* cnt = is_x ? S.nxl : S.nyl;
  const uint32_t j = atomicAdd(&cnt[sg], 1u);
  if (j >= P.seg_cap) { atomicOr(S.err, GG_DERR_CAP); return; }
  (is_x ? S.xl : S.yl)[(size_t)sg * P.seg_cap + j] = (uint64_t)r | ((uint64_t)m.dst << 32);
}

// ---- launchers (gg_coh_step.hip, gg_coh_persist.hip, gg_coh_walk.hip) ----
// k_c_step's arguments: the device copies of the launch state and this launch's timing slot
struct StepArgs { const CP* P; const CS* S; unsigned long long* kt; uint32_t kt_slot; };
void launch_step(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier);
void launch_step_fast(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier);
hipError_t step_fast_set_lds(size_t lds);
void launch_step_mosi(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier);
hipError_t step_mosi_set_lds(size_t lds);
void launch_step_shl2(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L, uint32_t devloop, uint64_t barrier);
hipError_t step_shl2_set_lds(size_t lds);
void launch_persist(bool lc, const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L0, uint32_t L1);
hipError_t step_set_lds(size_t step_lds, size_t persist_lc_lds, size_t persist_lds);
hipError_t persist_occupancy(bool lc, size_t lds, int* per_cu);
hipError_t persist_set_lds(size_t persist_lc_lds, size_t persist_lds);
void launch_persist_lc(const CP& P, const StepArgs& a, size_t lds, hipStream_t s, uint32_t L0, uint32_t L1);
hipError_t persist_lc_set_lds(size_t lds);
hipError_t persist_lc_occ(size_t lds, int* per_cu);
void launch_walk(bool pipe, bool rq, uint32_t blocks, uint32_t threads, size_t lds, hipStream_t s, const StepArgs& a,
                 uint32_t L, int stage);
hipError_t walk_set_lds(size_t lds);

}  // namespace ggc
