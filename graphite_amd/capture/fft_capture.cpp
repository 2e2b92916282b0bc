// fft_capture.cpp — trace-capture front end for BASELINE configs[0]
// ("SPLASH-2 FFT 16 tiles ... CPU reference w/ trace capture").
//
// The reference captures an application's memory operands with Pin
// (pin/lite/memory_modeling.cc:13-89) and feeds each one to
// Core::initiateMemoryAccess.  Pin is not available here, so the application
// is instrumented at the source level instead: a six-step 1-D FFT with the
// structure of SPLASH-2 FFT (tests/benchmarks/fft/fft.C: P threads, each
// owning rootN/P rows of the rootN x rootN matrix view; blocked transposes
// with padded rows; row FFTs with a private copy of the rootN roots of unity;
// twiddles from the full N-entry root matrix; barriers between phases) runs
// single-threadedly, phase by phase, and every 8-byte load and store it makes
// to the shared arrays is appended to the issuing thread's trace as one
// record of the graphite_gpu.h trace format:
//   addr = byte address in a fixed synthetic address map (below),
//   meta = WRITE bit | (gap << 1), gap = floating-point operations the thread
//          executed since its previous access (a 1-cycle-per-flop core).
// Thread t's records form tile t's trace.  Barriers are not modelled as
// records (the trace-driven path has no synchronisation records); phase
// order within a thread is preserved.
//
// C ABI (graphite_amd/capture.py binds it): gg_fft_capture_create / _counts /
// _copy / _output / _destroy.  Capture-side code: not on the GPU path.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

// synthetic address map (page-aligned arrays; rows padded as SPLASH-2 does)
constexpr uint64_t kBaseX = 0x10000000ull;        // x      : N complex + padding
constexpr uint64_t kBaseTrans = 0x50000000ull;    // trans  : N complex + padding
constexpr uint64_t kBaseU = 0x90000000ull;        // umain  : rootN complex (roots for 1-D FFTs)
constexpr uint64_t kBaseU2 = 0xA0000000ull;       // umain2 : N complex + padding (twiddle matrix)
constexpr uint64_t kBasePriv = 0xE0000000ull;     // upriv  : per-thread copy of umain, 1 MiB apart

struct Capture {
  uint32_t M, P;
  uint64_t N, n1, pad, row;                       // row = n1 + pad complex elements
  std::vector<double> x, trans, u, u2;
  std::vector<std::vector<double>> upriv;
  std::vector<std::vector<uint64_t>> addr;
  std::vector<std::vector<uint32_t>> meta;
  std::vector<uint64_t> flops;                    // per thread, since its last access

  void rec(uint32_t t, uint64_t a, bool w)
  {
    const uint64_t gap = flops[t] > 0x3FFFFFFFull ? 0x3FFFFFFFull : flops[t];
    addr[t].push_back(a);
    meta[t].push_back((uint32_t)((gap << 1) | (w ? 1u : 0u)));
    flops[t] = 0;
  }
  // complex element access helpers: re then im, 8 B each
  void ld(uint32_t t, uint64_t base, uint64_t idx) { rec(t, base + idx * 16, false); rec(t, base + idx * 16 + 8, false); }
  void st(uint32_t t, uint64_t base, uint64_t idx) { rec(t, base + idx * 16, true); rec(t, base + idx * 16 + 8, true); }
  uint64_t mi(uint64_t r, uint64_t c) const { return r * row + c; }   // padded matrix index

  // Blocked transpose of thread t's rows of dst (columns of src): dst[r][c] = src[c][r].
  // Staggered as SPLASH-2 does: thread t starts with the column block of its
  // own rows, so threads read different blocks at the same time.
  void transpose(uint32_t t, std::vector<double>& src, uint64_t sbase, std::vector<double>& dst, uint64_t dbase)
  {
    const uint64_t rows = n1 / P, r0 = t * rows;
    const uint64_t blk = rows < 8 ? rows : 8;
    for (uint64_t k = 0; k < P; ++k) {
      const uint64_t cb = ((t + k) % P) * rows;   // column block
      for (uint64_t rb = 0; rb < rows; rb += blk)
        for (uint64_t cc = 0; cc < rows; cc += blk)
          for (uint64_t r = r0 + rb; r < r0 + rb + blk; ++r)
            for (uint64_t c = cb + cc; c < cb + cc + blk; ++c) {
              ld(t, sbase, mi(c, r));
              dst[2 * mi(r, c)] = src[2 * mi(c, r)];
              dst[2 * mi(r, c) + 1] = src[2 * mi(c, r) + 1];
              st(t, dbase, mi(r, c));
            }
    }
  }

  // In-place radix-2 FFT of one row (length n1) with thread t's private roots.
  void fft_row(uint32_t t, std::vector<double>& a, uint64_t base, uint64_t r, int dir)
  {
    const uint64_t o = mi(r, 0);
    const uint32_t m = M / 2;
    // bit reversal
    for (uint64_t i = 0; i < n1; ++i) {
      uint64_t j = 0;
      for (uint32_t b = 0; b < m; ++b) j |= ((i >> b) & 1u) << (m - 1 - b);
      if (j > i) {
        ld(t, base, o + i); ld(t, base, o + j);
        std::swap(a[2 * (o + i)], a[2 * (o + j)]);
        std::swap(a[2 * (o + i) + 1], a[2 * (o + j) + 1]);
        st(t, base, o + i); st(t, base, o + j);
      }
    }
    const std::vector<double>& up = upriv[t];
    const uint64_t pbase = kBasePriv + (uint64_t)t * (1ull << 20);
    for (uint64_t len = 2; len <= n1; len <<= 1) {
      const uint64_t half = len / 2, stride = n1 / len;
      for (uint64_t s = 0; s < n1; s += len)
        for (uint64_t k = 0; k < half; ++k) {
          const uint64_t wi = k * stride;                  // W_n1^(k*stride)
          ld(t, pbase, wi);
          const double wr = up[2 * wi], wim = dir * up[2 * wi + 1];
          const uint64_t i0 = o + s + k, i1 = i0 + half;
          ld(t, base, i0); ld(t, base, i1);
          const double xr = a[2 * i1] * wr - a[2 * i1 + 1] * wim;
          const double xi = a[2 * i1] * wim + a[2 * i1 + 1] * wr;
          const double yr = a[2 * i0], yi = a[2 * i0 + 1];
          a[2 * i0] = yr + xr; a[2 * i0 + 1] = yi + xi;
          a[2 * i1] = yr - xr; a[2 * i1 + 1] = yi - xi;
          flops[t] += 10;
          st(t, base, i0); st(t, base, i1);
        }
    }
  }

  // trans[r][c] *= W_N^(r*c) from umain2 (thread t's rows)
  void twiddle(uint32_t t, int dir)
  {
    const uint64_t rows = n1 / P;
    for (uint64_t r = t * rows; r < (t + 1) * rows; ++r)
      for (uint64_t c = 0; c < n1; ++c) {
        const uint64_t i = mi(r, c);
        ld(t, kBaseU2, i);
        ld(t, kBaseTrans, i);
        const double wr = u2[2 * i], wim = dir * u2[2 * i + 1];
        const double ar = trans[2 * i], ai = trans[2 * i + 1];
        trans[2 * i] = ar * wr - ai * wim;
        trans[2 * i + 1] = ar * wim + ai * wr;
        flops[t] += 6;
        st(t, kBaseTrans, i);
      }
  }

  void run(int dir)
  {
    // each phase runs for every thread before the next (barriers)
    for (uint32_t t = 0; t < P; ++t) transpose(t, x, kBaseX, trans, kBaseTrans);
    for (uint32_t t = 0; t < P; ++t)
      for (uint64_t r = t * (n1 / P); r < (t + 1) * (n1 / P); ++r) fft_row(t, trans, kBaseTrans, r, dir);
    for (uint32_t t = 0; t < P; ++t) twiddle(t, dir);
    for (uint32_t t = 0; t < P; ++t) transpose(t, trans, kBaseTrans, x, kBaseX);
    for (uint32_t t = 0; t < P; ++t)
      for (uint64_t r = t * (n1 / P); r < (t + 1) * (n1 / P); ++r) fft_row(t, x, kBaseX, r, dir);
    for (uint32_t t = 0; t < P; ++t) transpose(t, x, kBaseX, trans, kBaseTrans);
  }
};

}  // namespace

extern "C" {

// Forward FFT of 2^m points on p threads (m even, p a power of two dividing
// 2^(m/2)); input x[j] = (sin(j) + 0.1 j mod 1, cos(j / 3)) (deterministic).
// Returns NULL on a bad argument.
void* gg_fft_capture_create(uint32_t m, uint32_t p)
{
  if (m < 2 || (m & 1) || m > 24 || p == 0 || (p & (p - 1))) return nullptr;
  const uint64_t n1 = 1ull << (m / 2);
  if (p > n1) return nullptr;
  Capture* c = new Capture;
  c->M = m; c->P = p; c->N = 1ull << m; c->n1 = n1;
  c->pad = 64 / 16;                                   // one 64-B line of padding per row (SPLASH-2 pads rows)
  c->row = n1 + c->pad;
  const uint64_t cells = n1 * c->row;
  c->x.assign(2 * cells, 0.0); c->trans.assign(2 * cells, 0.0);
  c->u.assign(2 * n1, 0.0); c->u2.assign(2 * cells, 0.0);
  c->upriv.assign(p, std::vector<double>());
  c->addr.assign(p, {}); c->meta.assign(p, {}); c->flops.assign(p, 0);
  for (uint64_t j = 0; j < c->N; ++j) {
    const uint64_t r = j / n1, col = j % n1;
    c->x[2 * c->mi(r, col)] = std::sin((double)j) + std::fmod(0.1 * (double)j, 1.0);
    c->x[2 * c->mi(r, col) + 1] = std::cos((double)j / 3.0);
  }
  const double pi = 3.14159265358979323846;
  for (uint64_t k = 0; k < n1; ++k) {
    c->u[2 * k] = std::cos(2 * pi * (double)k / (double)n1);
    c->u[2 * k + 1] = -std::sin(2 * pi * (double)k / (double)n1);
  }
  for (uint64_t r = 0; r < n1; ++r)
    for (uint64_t col = 0; col < n1; ++col) {
      const double a = 2 * pi * (double)(r * col) / (double)c->N;
      c->u2[2 * c->mi(r, col)] = std::cos(a);
      c->u2[2 * c->mi(r, col) + 1] = -std::sin(a);
    }
  // each thread copies the 1-D roots into its private array (recorded)
  for (uint32_t t = 0; t < p; ++t) {
    c->upriv[t] = c->u;
    for (uint64_t k = 0; k < n1; ++k) {
      c->ld(t, kBaseU, k);
      c->st(t, kBasePriv + (uint64_t)t * (1ull << 20), k);
    }
  }
  c->run(1);
  return c;
}

// Records per thread (p entries).
void gg_fft_capture_counts(void* h, uint64_t* counts)
{
  Capture* c = (Capture*)h;
  for (uint32_t t = 0; t < c->P; ++t) counts[t] = c->addr[t].size();
}

// Thread-major trace (the graphite_gpu.h gg_trace layout).
void gg_fft_capture_copy(void* h, uint64_t* addr, uint32_t* meta)
{
  Capture* c = (Capture*)h;
  uint64_t o = 0;
  for (uint32_t t = 0; t < c->P; ++t) {
    std::memcpy(addr + o, c->addr[t].data(), c->addr[t].size() * 8);
    std::memcpy(meta + o, c->meta[t].data(), c->meta[t].size() * 4);
    o += c->addr[t].size();
  }
}

// The transform's result, X[k] as (re, im) pairs, natural order (2N doubles).
void gg_fft_capture_output(void* h, double* out)
{
  Capture* c = (Capture*)h;
  for (uint64_t k = 0; k < c->N; ++k) {
    const uint64_t r = k / c->n1, col = k % c->n1;
    out[2 * k] = c->trans[2 * c->mi(r, col)];
    out[2 * k + 1] = c->trans[2 * c->mi(r, col) + 1];
  }
}

// The input, x[j] as (re, im) pairs (2N doubles).
void gg_fft_capture_input(uint32_t m, double* out)
{
  const uint64_t N = 1ull << m;
  for (uint64_t j = 0; j < N; ++j) {
    out[2 * j] = std::sin((double)j) + std::fmod(0.1 * (double)j, 1.0);
    out[2 * j + 1] = std::cos((double)j / 3.0);
  }
}

void gg_fft_capture_destroy(void* h) { delete (Capture*)h; }

}  // extern "C"
