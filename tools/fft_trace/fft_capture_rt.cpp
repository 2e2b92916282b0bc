// fft_capture_rt.cpp — trace capture runtime for the reference's SPLASH-2 FFT
// (tests/benchmarks/fft/fft.C), standing in for Graphite's Pin front end
// (pin/lite/memory_modeling.cc:13-89: every memory operand of a modeled
// thread becomes a Core::initiateMemoryAccess on its tile).
//
// fft.C is compiled with -fsanitize=thread, which makes the compiler call
// __tsan_readN / __tsan_writeN(address) before every memory access it cannot
// prove thread-private; this file defines those hooks (the TSan runtime is
// not linked) and appends each access to the issuing thread's trace while
// the models are enabled (CarbonEnableModels .. CarbonDisableModels around
// CREATE / WAIT_FOR_END, fft.C:323-330).  Thread k (ProcID k) is tile k.
// Only heap accesses are recorded: every allocation comes from one arena
// (the main thread's in allocation order, each thread's in a region of its
// own), and an access's address is rebased to kCanon + its arena offset, so
// the trace does not depend on ASLR, malloc or thread timing; the program's scalar globals and
// stack (registers at -O2, or thread-private) are not.
// Record: addr u64, meta u32 = WRITE | (gap << 1) with gap = 1 core cycle
// (the instructions between memory operands are not observed; one cycle
// each is the trace's timing model).  BARRIER(...) records the position
// in the thread's trace (the replayer does not model barriers).
//
// Output (GG_FFT_TRACE_OUT): "GGFT" u32 version=1 u32 P, u64 count[P],
// u64 nbar[P], then per tile addr[count] u64 and meta[count] u32, then per
// tile barrier positions u64[nbar].  Capture tool only, never on the GPU path.
#include <pthread.h>
#include <sys/mman.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

constexpr uint64_t kCanon = 0x100000000ull;             // canonical address of arena offset 0
constexpr size_t kArenaBytes = (size_t)8 << 30;         // reserved, not committed
constexpr size_t kSharedBytes = (size_t)4 << 30;        // allocations before CREATE (main thread)
constexpr size_t kTileBytes = (size_t)4 << 20;          // per-thread allocations inside the threads (upriv)
constexpr uint32_t kGapCycles = 1;

char* g_arena = nullptr;
size_t g_used = 0;                                      // shared region (single-threaded)
size_t g_tile_used[1024];                               // per-thread regions: allocation order is per thread
std::atomic<bool> g_on{false};
std::atomic<long> g_turn{0};
long g_P = 0;
pthread_barrier_t g_bar;
pthread_t g_th[1024];
std::vector<uint64_t>* g_addr = nullptr;
std::vector<uint32_t>* g_meta = nullptr;
std::vector<uint64_t>* g_bars = nullptr;
thread_local long t_tile = -1;

inline void rec(const void* p, bool w)
{
  if (t_tile < 0 || !g_on.load(std::memory_order_relaxed)) return;
  const uint64_t off = (uint64_t)((const char*)p - g_arena);
  if (off >= kArenaBytes) return;
  g_addr[t_tile].push_back(kCanon + off);
  g_meta[t_tile].push_back((kGapCycles << 1) | (w ? 1u : 0u));
}

struct Start { void (*fn)(void); long tile; };
Start g_start[1024];

void* thread_main(void* arg)
{
  Start* s = (Start*)arg;
  t_tile = s->tile;
  s->fn();
  return nullptr;
}

}  // namespace

extern "C" {

void __tsan_init(void) {}
void __tsan_func_entry(void*) {}
void __tsan_func_exit(void) {}
void __tsan_read1(void* p) { rec(p, false); }
void __tsan_read2(void* p) { rec(p, false); }
void __tsan_read4(void* p) { rec(p, false); }
void __tsan_read8(void* p) { rec(p, false); }
void __tsan_read16(void* p) { rec(p, false); }
void __tsan_write1(void* p) { rec(p, true); }
void __tsan_write2(void* p) { rec(p, true); }
void __tsan_write4(void* p) { rec(p, true); }
void __tsan_write8(void* p) { rec(p, true); }
void __tsan_write16(void* p) { rec(p, true); }

void* gg_cap_malloc(size_t n)
{
  if (!g_arena) {
    void* a = mmap(nullptr, kArenaBytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (a == MAP_FAILED) { perror("gg_cap_malloc"); exit(2); }
    g_arena = (char*)a;
  }
  // 64-B aligned blocks in allocation order: the main thread's before
  // CREATE in the shared region, each thread's own in its region (threads
  // allocate concurrently, so one bump pointer would order them by timing)
  const size_t sz = (n + 63) & ~(size_t)63;
  size_t at;
  if (t_tile < 0) {
    at = g_used; g_used += sz;
    if (g_used > kSharedBytes) { fprintf(stderr, "gg_cap_malloc: arena exhausted\n"); exit(2); }
  } else {
    if (t_tile >= (long)((kArenaBytes - kSharedBytes) / kTileBytes) || g_tile_used[t_tile] + sz > kTileBytes) {
      fprintf(stderr, "gg_cap_malloc: thread region exhausted\n"); exit(2);
    }
    at = kSharedBytes + (size_t)t_tile * kTileBytes + g_tile_used[t_tile];
    g_tile_used[t_tile] += sz;
  }
  return g_arena + at;
}

void gg_cap_create(void (*fn)(void), long p)
{
  if (p < 1 || p > 1024) { fprintf(stderr, "gg_cap_create: P = %ld\n", p); exit(2); }
  g_P = p;
  g_addr = new std::vector<uint64_t>[p];
  g_meta = new std::vector<uint32_t>[p];
  g_bars = new std::vector<uint64_t>[p];
  t_tile = 0;
  for (long i = 1; i < p; ++i) {
    g_start[i] = Start{fn, i};
    if (pthread_create(&g_th[i], nullptr, thread_main, &g_start[i])) { fprintf(stderr, "pthread_create\n"); exit(2); }
  }
  fn();
}

void gg_cap_wait(long p)
{
  for (long i = 1; i < p; ++i) pthread_join(g_th[i], nullptr);
}

// fft.C's one lock hands out ProcIDs (SlaveStart, fft.C:437-440): threads take
// it in tile order, so thread k gets ProcID k
void gg_cap_lock(pthread_mutex_t* l)
{
  const long me = t_tile < 0 ? 0 : t_tile;
  while (g_turn.load() != me) sched_yield();
  pthread_mutex_lock(l);
}

void gg_cap_unlock(pthread_mutex_t* l)
{
  pthread_mutex_unlock(l);
  g_turn.fetch_add(1);
}

void gg_cap_barrier_init(long n) { pthread_barrier_init(&g_bar, nullptr, (unsigned)n); }

void gg_cap_barrier(void)
{
  if (t_tile >= 0 && g_bars) g_bars[t_tile].push_back(g_addr[t_tile].size());
  pthread_barrier_wait(&g_bar);
}

void CarbonEnableModels(void) { g_on = true; }

void CarbonDisableModels(void)
{
  g_on = false;
  const char* path = getenv("GG_FFT_TRACE_OUT");
  if (!path || !g_addr) return;
  FILE* f = fopen(path, "wb");
  if (!f) { perror(path); exit(2); }
  const uint32_t hdr[3] = {0x54464747u, 1u, (uint32_t)g_P};   // "GGFT"
  fwrite(hdr, sizeof hdr, 1, f);
  for (long t = 0; t < g_P; ++t) { const uint64_t c = g_addr[t].size(); fwrite(&c, 8, 1, f); }
  for (long t = 0; t < g_P; ++t) { const uint64_t c = g_bars[t].size(); fwrite(&c, 8, 1, f); }
  for (long t = 0; t < g_P; ++t) {
    fwrite(g_addr[t].data(), 8, g_addr[t].size(), f);
    fwrite(g_meta[t].data(), 4, g_meta[t].size(), f);
  }
  for (long t = 0; t < g_P; ++t) fwrite(g_bars[t].data(), 8, g_bars[t].size(), f);
  fclose(f);
}

}  // extern "C"
