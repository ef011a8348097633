// photon_ml_amd — CDNA4 (gfx950 / MI355X) fused per-entity PRIMAL TRON for random effects.
//
// The reference solves every random-effect entity as its own small GLM (photon-api/.../algorithm/
// RandomEffectCoordinate.scala:103-143 -> optimization/SingleNodeOptimizationProblem.scala:85-103 -> photon-lib/
// .../optimization/TRON.scala:80-340). Entities with few rows are solved in their row space (rs_tron in
// glm_kernels.hip); this file handles the others — typically 65 .. thousands of rows over ~1k projected
// coefficients — WITHOUT a pass-per-Hessian-vector launch sequence over the whole block-diagonal problem:
//
// * one workgroup (4 waves) owns one entity for its whole solve: the coefficient-space vectors (w, g, step, r,
//   d) and one accumulator per wave live in LDS (d_e <= dmax doubles each); the TRON control flow (truncated CG,
//   trust-region radius, accept / reject, Photon convergence tests) runs on workgroup-uniform scalars;
// * every Hessian-vector product X^T (D (X d)) is ONE read of the entity's CSR rows (a wave per row, lane k =
//   non-zero k of the row: gather d[c] from LDS, DPP wave sum, scale by the cached D_i = w_i l''(z_i), scatter
//   t x_ik into the wave's private LDS accumulator). The block-diagonal pass path reads the rows twice (CSR
//   forward + CSC transpose copy) per product and launches per pass; here there is no CSC copy at all;
// * deterministic: fixed-order DPP / readlane wave sums, per-wave accumulators combined in wave order, distinct
//   columns inside a row (so one ds_add_f64 never has two lanes on one address within a row);
// * per-row scratch in HBM: D and the margins x_i.w for the current iterate and the trial point (swapped on
//   acceptance), so the final margins come out of the solve (scores without another pass).
//
// Semantics follow batched_tron / rs_tron_kernel: eta = (1e-4, .25, .75), sigma = (.25, .5, 4), delta0 = ||g0||,
// first-iteration delta = min(delta, ||step||), CG tolerance 0.1 ||g||, <= max_cg CG steps, <= max_fail
// consecutive rejections; reason codes 1 max-iter, 2 not-improving, 3 f-converged, 4 g-converged; tolerances
// from the state at zero coefficients (photon-lib/.../optimization/Optimizer.scala:136-196).
//
// Built with: hipcc --offload-arch=gfx950 -O3 -shared -fPIC (photon_ml_amd/ops/build.py). C ABI, ctypes.

#include <hip/hip_runtime.h>
#include <stdint.h>

// Build id (photon_ml_amd/ops/build.py: content hash of the sources + compile command, -DPML_BUILD_ID=...): the
// loaders compare it with the tree's sources and refuse a stale library.
#ifndef PML_BUILD_ID
#define PML_BUILD_ID "unstamped-build!"
#endif
__attribute__((used)) static const char pml_build_stamp[] = "PML_BUILD_ID=" PML_BUILD_ID;

#define LAUNCH_CHECK()                                         \
  do {                                                         \
    hipError_t e_ = hipGetLastError();                         \
    if (e_ != hipSuccess) return (int)e_;                      \
  } while (0)

#define RE_NW 4                 // waves per workgroup (one entity)
#define RE_THREADS (RE_NW * 64)

enum { LOSS_LOGISTIC = 0, LOSS_POISSON = 1, LOSS_SQUARED = 2 };

template <int LOSS>
__device__ __forceinline__ void loss_t(double z, double y, double& l, double& dl, double& d2) {
  if constexpr (LOSS == LOSS_LOGISTIC) {
    // one exp, one log1p, one reciprocal, no branches (as pointwise_loss in glm_kernels.hip):
    // e = exp(-|z|) serves the sigmoid and log(1 + exp(+-z)) = max(+-z, 0) + log1p(e)
    const double e = exp(-fabs(z));
    const double lp = log1p(e);
    const double r = 1.0 / (1.0 + e);
    const double s = z >= 0.0 ? r : e * r;
    const bool pos = y > 0.5;
    const double zz = pos ? -z : z;
    l = (zz > 0.0 ? zz : 0.0) + lp;
    dl = pos ? s - 1.0 : s;
    d2 = s * (1.0 - s);
  } else if constexpr (LOSS == LOSS_POISSON) {
    const double e = exp(z);
    l = e - y * z; dl = e - y; d2 = e;
  } else {
    const double d = z - y;
    l = 0.5 * d * d; dl = d; d2 = 1.0;
  }
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned int)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned int)lo);
}

// Sum over the 64 lanes of a wave, returned (bitwise identical) in every lane: DPP butterflies inside each
// 16-lane row (every lane then holds its row's sum), then the four row sums in a fixed order.
__device__ __forceinline__ double wave_total(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// A workgroup-uniform value re-tagged as wave-uniform (readfirstlane): it is held in SGPRs, not VGPRs.
__device__ __forceinline__ long long uniform_i64(long long v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)v);
  const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
  return ((long long)hi << 32) | (long long)(unsigned int)lo;
}
__device__ __forceinline__ double uniform_f64(double v) {
  return __builtin_bit_cast(double, uniform_i64(__builtin_bit_cast(long long, v)));
}

// Workgroup sums of K values (K <= 8), in every thread. ``red`` holds two [RE_NW][8] slots used alternately,
// so one barrier per call suffices: a slot is rewritten only two calls later, after every thread has passed
// the barrier of the call in between (all threads run the same, workgroup-uniform control flow).
template <int K, int NW = RE_NW>
__device__ __forceinline__ void block_sums(double (&v)[K], double* __restrict__ red, int& parity) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_total(v[k]);
  double* slot = red + parity * (NW * 8);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) slot[w * 8 + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += slot[q * 8 + k];
    v[k] = uniform_f64(s);      // identical in every thread
  }
  parity ^= 1;
}

struct ReTronArgs {
  const int* order;          // launch slot -> entity (largest entities first)
  int n_launch;
  const long long* row_ptr;  // [E + 1] entity row ranges
  const long long* col_ptr;  // [E + 1] entity coefficient ranges (packed W)
  const long long* nip;      // [N + 1] row -> non-zero range
  const uint16_t* lcol;      // entity-local column of every non-zero (< d_e, distinct inside a row)
  const double* val;         // value of every non-zero
  const double* y;           // per-row label / offset / weight
  const double* off;
  const double* wt;
  double* scr;               // per-row scratch [4][n_rows]: D (2 buffers), margins x.w (2 buffers)
  long long n_rows;
  double* W;                 // packed coefficients: in = warm start, out = solution
  double* f;                 // per entity: final objective, iterations, reason code
  int* iters;
  int* reason;
  double* zout;              // per row: x_i . w of the solution (no offset)
  int* npass;                // optional, per entity: row passes run (function evaluations + Hessian-vector)
  int loss;
  double l2, tol;
  int max_iter, max_fail, max_cg, dmax;
  double* gsc;               // lean kernel: gradient at W, per coefficient (packed like W)
  const double* xf2;         // lean kernel, optional: ||X_e||_F^2 per entity (lazy zero-point gradient norm)
};

// Loads through the global address space: a generic pointer read through the kernel-argument struct becomes a FLAT
// load, which also counts in lgkmcnt -- every LDS wait would then wait for it too.
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}

// Sum over the 16 lanes of a DPP row, in every lane of the row (fixed-order butterflies: deterministic).
__device__ __forceinline__ double row16_total(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
  return v;
}

#define RE_G 16                      // lanes per row (one DPP row)
#define RE_RPI (64 / RE_G)           // rows per wave instruction
#define RE_U 4                       // row groups in flight per wave batch (re_tron_csr_kernel; 3: +2.4 %)
#define RE_K 4                       // entries per lane kept in registers (rows of <= 64 entries in one go)
#ifndef RE_ABL
#define RE_ABL 0                     // profiling-only ablation mask (see row_pass); 0 in production
#endif

// One pass over the entity's rows [r0, r1): a wave takes BATCH = 4 U consecutive rows at a time, RE_G lanes per
// row (lane k of the row: entries k, k + 16, ...). The next batch's row pointers are fetched while the current
// batch computes, and all BATCH rows' entries are loaded before the first gather, so a batch costs about one
// dependent global-memory latency.
// MODE 0: Hessian-vector data term: acc_w += X^T (Dc * (X vec)).
// MODE 1: value + gradient at vec: acc_w += X^T (wt * l'), fpart += wt * l, Dn = wt * l'', Zn = x.vec.
// MODE 2: value + gradient at zero (no gathers, no scratch writes).
template <int MODE, int LOSS, int U = RE_U, int NW = RE_NW>
__device__ __forceinline__ void row_pass(const ReTronArgs& a, long long r0, long long r1,
                                         const double* __restrict__ vec, double* __restrict__ acc,
                                         const double* __restrict__ Dc, double* __restrict__ Dn,
                                         double* __restrict__ Zn, double& fpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / RE_G, gl = lane % RE_G;
  // entity-local 32-bit row / entry offsets from per-entity bases: one VGPR per address instead of 64-bit math
  const int nrows = (int)(r1 - r0);
  const long long e0 = a.nip[r0];
  const long long* __restrict__ nip = a.nip + r0;
  const uint16_t* __restrict__ lcol = a.lcol + e0;
  const double* __restrict__ val = a.val + e0;
  const double* __restrict__ wt = a.wt + r0;
  const double* __restrict__ off = a.off + r0;
  const double* __restrict__ yv = a.y + r0;
  if (MODE == 0) Dc += r0;
  if (MODE == 1) { Dn += r0; Zn += r0; }
  constexpr int BATCH = RE_RPI * U;
  const int step = NW * BATCH;
  int base = w * BATCH;
  // row pointers of a batch, prefetched one batch ahead: lane j <= BATCH holds nip[base + j] (clamped to the
  // entity's end). The load is unconditional and its raw value is only converted at its use in the next batch, so
  // the prefetch never waits (a conditional load / immediate conversion put a full memory round trip per batch)
  auto fetch_raw = [&](int b) -> long long {
    const int i = b + (lane <= BATCH ? lane : BATCH);
    return gld(nip + (i < nrows ? i : nrows));
  };
  long long npr = fetch_raw(base);
  for (; base < nrows; base += step) {
    const int np = (int)(npr - e0);
    const long long npr_next = fetch_raw(base + step);
    int lo[U], hi[U];
    int c[U][RE_K];
    double v[U][RE_K], dot[U], rs[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = u * RE_RPI + grp;
      lo[u] = __shfl(np, q, 64);
      hi[u] = __shfl(np, q + 1, 64);
      const int i = base + q;
      const bool valid = i < nrows;
      const int ic = valid ? i : 0;
      if (MODE == 0) {
        rs[u][0] = valid ? gld(Dc + ic) : 0.0;
      } else {
        rs[u][0] = valid ? gld(wt + ic) : 0.0;
        rs[u][1] = valid ? gld(off + ic) : 0.0;
        rs[u][2] = valid ? gld(yv + ic) : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < RE_K; ++k) {
        const int p = lo[u] + gl + RE_G * k;
        const bool in = p < hi[u];
        c[u][k] = in ? (int)lcol[p] : 0;
        v[u][k] = in ? val[p] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double s = 0.0;
      if (MODE != 2) {
#pragma unroll
        for (int k = 0; k < RE_K; ++k) s = fma(v[u][k], vec[c[u][k]], s);
        for (int p = lo[u] + gl + RE_G * RE_K; p < hi[u]; p += RE_G) s = fma(val[p], vec[lcol[p]], s);
#if RE_ABL
        // profiling ablations (scripts/gpu_r5_s5.sh): the same math plus one extra LDS gather (2) or one extra
        // value load (4) per entry, scaled by a runtime zero -- their marginal cost, at identical iterates
        const double zero = a.l2 - a.l2;
#pragma unroll
        for (int k = 0; k < RE_K; ++k) {
          if (RE_ABL & 2) s = fma(zero, vec[c[u][k] >> 1], s);
          if (RE_ABL & 4) {
            const int p = lo[u] + gl + RE_G * k;
            s = fma(zero, p < hi[u] ? ((volatile const double*)val)[p] : 0.0, s);
          }
        }
#endif
      }
      dot[u] = s;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE != 2) dot[u] = row16_total(dot[u]);
      const int i = base + u * RE_RPI + grp;
      const bool valid = i < nrows;
      double t;
      if (MODE == 0) {
        t = rs[u][0] * dot[u];
      } else {
        double l = 0.0, dl = 0.0, d2 = 0.0;
        if (valid) {
          loss_t<LOSS>(dot[u] + rs[u][1], rs[u][2], l, dl, d2);
          if (gl == 0) {
            fpart += rs[u][0] * l;
            if (MODE == 1) { Dn[i] = rs[u][0] * d2; Zn[i] = dot[u]; }
          }
        }
        t = rs[u][0] * dl;
      }
#pragma unroll
      for (int k = 0; k < RE_K; ++k)
        if (lo[u] + gl + RE_G * k < hi[u]) {
          atomicAdd(&acc[c[u][k]], t * v[u][k]);
#if RE_ABL & 1
          atomicAdd(&acc[c[u][k]], (a.l2 - a.l2) * v[u][k]);   // profiling: one extra LDS atomic per entry
#endif
        }
      for (int p = lo[u] + gl + RE_G * RE_K; p < hi[u]; p += RE_G) atomicAdd(&acc[lcol[p]], t * val[p]);
    }
    npr = npr_next;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Quad row pass (lean kernel, rows padded to whole quads of 4 entries: EntityTronBatch pads with column 0 / value
// 0.0, which add exactly nothing). Lane gl of a row's 16 lanes owns the quad gl (+ 16 per extra chunk): its 4
// columns arrive in ONE 8-byte load and its 4 values in TWO 16-byte loads, where row_pass issues 4 + 4 narrow
// loads. The kernel is bound by the texture path's per-instruction work (profiles/re_lean_ablation_r5.md: one
// extra value load per entry costs +67 %, one extra LDS atomic +8 %), so 3 instead of 8 loads per 4 entries.
// Only a quad past the row end is masked (no per-entry masks).
typedef double re_d2 __attribute__((ext_vector_type(2)));
typedef unsigned re_u2 __attribute__((ext_vector_type(2)));

// Four LDS gathers in flight together (one wait for all four): left to itself the compiler issues each gather,
// waits for it and consumes it before the next (register pressure), which serialises four LDS round trips per
// lane per row group. ``vec`` is a __shared__ array; the byte offsets are its LDS addresses.
__device__ __forceinline__ void lds_gather4(const double* vec, int c0, int c1, int c2, int c3, double& g0, double& g1,
                                            double& g2, double& g3) {
  const unsigned b = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) double*)vec;
  const unsigned a0 = b + 8u * (unsigned)c0, a1 = b + 8u * (unsigned)c1, a2 = b + 8u * (unsigned)c2,
                 a3 = b + 8u * (unsigned)c3;
  asm volatile(
      "ds_read_b64 %0, %4\n\t"
      "ds_read_b64 %1, %5\n\t"
      "ds_read_b64 %2, %6\n\t"
      "ds_read_b64 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(g0), "=&v"(g1), "=&v"(g2), "=&v"(g3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
      : "memory");
}

template <int MODE, int LOSS, int U, int NW = RE_NW>
__device__ __forceinline__ void row_pass_q(const ReTronArgs& a, long long r0, long long r1,
                                           const double* __restrict__ vec, double* __restrict__ acc,
                                           const double* __restrict__ Dc, double* __restrict__ Dn,
                                           double* __restrict__ Zn, double& fpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / RE_G, gl = lane % RE_G;
  const int nrows = (int)(r1 - r0);
  const long long e0 = a.nip[r0];                           // a multiple of 4 (padded rows)
  const long long* __restrict__ nip = a.nip + r0;
  const re_u2* __restrict__ cq = (const re_u2*)(a.lcol + e0);   // quad q: 4 columns
  const re_d2* __restrict__ vq = (const re_d2*)(a.val + e0);    // quad q: values at 2q, 2q + 1
  const double* __restrict__ wt = a.wt + r0;
  const double* __restrict__ off = a.off + r0;
  const double* __restrict__ yv = a.y + r0;
  if (MODE == 0) Dc += r0;
  if (MODE == 1) { Dn += r0; Zn += r0; }
  constexpr int BATCH = RE_RPI * U;
  const int step = NW * BATCH;
  int base = w * BATCH;
  // row pointers of a batch, in quads: lane j <= BATCH holds nip[base + j] / 4 (prefetched as in row_pass)
  auto fetch_raw = [&](int b) -> long long {
    const int i = b + (lane <= BATCH ? lane : BATCH);
    return gld(nip + (i < nrows ? i : nrows));
  };
  auto cols = [](re_u2 c, int (&k)[4]) {
    k[0] = (int)(c.x & 0xFFFFu); k[1] = (int)(c.x >> 16); k[2] = (int)(c.y & 0xFFFFu); k[3] = (int)(c.y >> 16);
  };
  long long npr = fetch_raw(base);
  for (; base < nrows; base += step) {
    const int np = (int)((npr - e0) >> 2);
    const long long npr_next = fetch_raw(base + step);
    int qa[U], qb[U];
    re_u2 c[U];
    re_d2 v0[U], v1[U];
    double dot[U], rs[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = u * RE_RPI + grp;
      qa[u] = __shfl(np, q, 64) + gl;                         // this lane's quad
      qb[u] = __shfl(np, q + 1, 64);                          // the row's end (quads)
      const int i = base + q;
      const bool valid = i < nrows;
      const int ic = valid ? i : 0;
      if (MODE == 0) {
        rs[u][0] = valid ? gld(Dc + ic) : 0.0;
      } else {
        rs[u][0] = valid ? gld(wt + ic) : 0.0;
        rs[u][1] = valid ? gld(off + ic) : 0.0;
        rs[u][2] = valid ? gld(yv + ic) : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = qa[u] < qb[u];
      const int qq = in ? qa[u] : 0;
      c[u] = gld(cq + qq);
      v0[u] = gld(vq + 2 * qq);
      v1[u] = gld(vq + 2 * qq + 1);
      if (!in) { c[u] = re_u2{0u, 0u}; v0[u] = re_d2{0.0, 0.0}; v1[u] = re_d2{0.0, 0.0}; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double s = 0.0;
      if (MODE != 2) {
        int k[4];
        cols(c[u], k);
        double g[4];
        lds_gather4(vec, k[0], k[1], k[2], k[3], g[0], g[1], g[2], g[3]);
        s = fma(v0[u].x, g[0], s);
        s = fma(v0[u].y, g[1], s);
        s = fma(v1[u].x, g[2], s);
        s = fma(v1[u].y, g[3], s);
        for (int qq = qa[u] + RE_G; qq < qb[u]; qq += RE_G) {     // rows longer than 64 entries
          int kt[4];
          cols(cq[qq], kt);
          const re_d2 a0 = vq[2 * qq], a1 = vq[2 * qq + 1];
          s = fma(a0.x, vec[kt[0]], s);
          s = fma(a0.y, vec[kt[1]], s);
          s = fma(a1.x, vec[kt[2]], s);
          s = fma(a1.y, vec[kt[3]], s);
        }
      }
      dot[u] = s;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE != 2) dot[u] = row16_total(dot[u]);
      const int i = base + u * RE_RPI + grp;
      const bool valid = i < nrows;
      double t;
      if (MODE == 0) {
        t = rs[u][0] * dot[u];
      } else {
        double l = 0.0, dl = 0.0, d2 = 0.0;
        if (valid) {
          loss_t<LOSS>(dot[u] + rs[u][1], rs[u][2], l, dl, d2);
          if (gl == 0) {
            fpart += rs[u][0] * l;
            if (MODE == 1) { Dn[i] = rs[u][0] * d2; Zn[i] = dot[u]; }
          }
        }
        t = rs[u][0] * dl;
      }
      if (qa[u] < qb[u]) {
        int k[4];
        cols(c[u], k);
        atomicAdd(&acc[k[0]], t * v0[u].x);
        atomicAdd(&acc[k[1]], t * v0[u].y);
        atomicAdd(&acc[k[2]], t * v1[u].x);
        atomicAdd(&acc[k[3]], t * v1[u].y);
      }
      for (int qq = qa[u] + RE_G; qq < qb[u]; qq += RE_G) {
        int kt[4];
        cols(cq[qq], kt);
        const re_d2 a0 = vq[2 * qq], a1 = vq[2 * qq + 1];
        atomicAdd(&acc[kt[0]], t * a0.x);
        atomicAdd(&acc[kt[1]], t * a0.y);
        atomicAdd(&acc[kt[2]], t * a1.x);
        atomicAdd(&acc[kt[3]], t * a1.y);
      }
    }
    npr = npr_next;
  }
}

template <int LOSS>
__global__ __launch_bounds__(RE_THREADS) void re_tron_csr_kernel(ReTronArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int e = a.order[blockIdx.x];
  const long long r0 = a.row_ptr[e], r1 = a.row_ptr[e + 1];
  const long long c0 = a.col_ptr[e];
  const int d = (int)(a.col_ptr[e + 1] - c0);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int dm = a.dmax;
  double* sW = smem;
  double* sG = sW + dm;
  double* sS = sG + dm;     // CG step
  double* sR = sS + dm;     // CG residual
  double* sD = sR + dm;     // CG direction; trial point during the function evaluation
  double* acc = sD + dm;    // RE_NW accumulators; acc[0 .. d) = combined Hd (with l2 d) / trial gradient
  double* red = acc + RE_NW * dm;
  double* myacc = acc + w * dm;
  double* D[2] = {a.scr, a.scr + a.n_rows};
  double* Z[2] = {a.scr + 2 * a.n_rows, a.scr + 3 * a.n_rows};
  int cur = 0, parity = 0, npass = 0;
  double* Wg = a.W + c0;

  auto zero_own = [&]() {
    for (int j = lane; j < d; j += 64) myacc[j] = 0.0;
  };
  // value + gradient at vec (MODE 1: writes D / Z buffer ``nb``); the gradient lands in acc[0 .. d). One sweep
  // combines the wave accumulators (fixed wave order) and forms ||vec||^2 and ||g||^2; three barriers in all.
  auto value_grad = [&](const double* vec, int nb, bool at_zero, double& gg) -> double {
    ++npass;
    __syncthreads();
    zero_own();
    double fp = 0.0;
    if (at_zero) row_pass<2, LOSS>(a, r0, r1, vec, myacc, nullptr, nullptr, nullptr, fp);
    else row_pass<1, LOSS>(a, r0, r1, vec, myacc, nullptr, D[nb], Z[nb], fp);
    __syncthreads();
    double s3[3] = {fp, 0.0, 0.0};
    for (int j = tid; j < d; j += RE_THREADS) {
      double g = acc[j];
#pragma unroll
      for (int q = 1; q < RE_NW; ++q) g += acc[q * dm + j];
      const double v = vec[j];
      g += a.l2 * v;
      acc[j] = g;
      s3[1] += v * v;
      s3[2] += g * g;
    }
    block_sums<3>(s3, red, parity);
    gg = s3[2];
    return s3[0] + 0.5 * a.l2 * s3[1];
  };

  for (int j = tid; j < d; j += RE_THREADS) sW[j] = Wg[j];
  double gnorm2;
  double f = value_grad(sW, cur, false, gnorm2);
  double nz[1] = {0.0};
  for (int j = tid; j < d; j += RE_THREADS) {
    sG[j] = acc[j];
    nz[0] += sW[j] != 0.0 ? 1.0 : 0.0;
  }
  block_sums<1>(nz, red, parity);
  double f0z = f, g0n = sqrt(gnorm2);
  if (nz[0] != 0.0) {
    for (int j = tid; j < d; j += RE_THREADS) sS[j] = 0.0;   // zero vector for the state at zero
    double g0;
    f0z = value_grad(sS, 0, true, g0);
    g0n = sqrt(g0);
  }
  const double loss_tol = f0z * a.tol, grad_tol = g0n * a.tol;
  double delta = sqrt(gnorm2);
  int it = 0, fails = 0, reason = 0;
  bool active = true;
  if (delta == 0.0) { reason = 4; active = false; }
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, sg1 = 0.25, sg2 = 0.5, sg3 = 4.0;
  const int guard_max = a.max_iter * (a.max_fail + 1) + 5;
  for (int guard = 0; active && guard < guard_max; ++guard) {
    // ---- truncated CG at W (Hessian weights D[cur]). Per CG step: the Hessian-vector pass, ONE sweep that
    // combines the accumulators and forms d.Hd, step.d, d.d, r.Hd, Hd.Hd, one workgroup sum, and one update
    // sweep; ||step + a d||^2 and ||r - a Hd||^2 follow by algebra (clamped at 0).
    for (int j = tid; j < d; j += RE_THREADS) {
      sS[j] = 0.0;
      sR[j] = -sG[j];
      sD[j] = -sG[j];
    }
    double rtr = gnorm2, sts = 0.0;
    const double cg_tol2 = 0.01 * gnorm2;        // (0.1 ||g||)^2
    for (int k = 0; k < a.max_cg; ++k) {
      if (!(rtr > cg_tol2)) break;
      ++npass;
      __syncthreads();
      zero_own();
      double fp = 0.0;
      row_pass<0, LOSS>(a, r0, r1, sD, myacc, D[cur], nullptr, nullptr, fp);
      __syncthreads();
      double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      for (int j = tid; j < d; j += RE_THREADS) {
        double h = acc[j];
#pragma unroll
        for (int q = 1; q < RE_NW; ++q) h += acc[q * dm + j];
        const double dj = sD[j];
        h += a.l2 * dj;
        acc[j] = h;
        s5[0] += dj * h;
        s5[1] += sS[j] * dj;
        s5[2] += dj * dj;
        s5[3] += sR[j] * h;
        s5[4] += h * h;
      }
      block_sums<5>(s5, red, parity);
      const double dhd = s5[0], std_ = s5[1], dtd = s5[2], rh = s5[3], hh = s5[4];
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      double tn = sts + 2.0 * alpha * std_ + alpha * alpha * dtd;
      tn = tn > 0.0 ? tn : 0.0;
      const double dsq = delta * delta;
      const bool hit = tn > dsq;
      double al = alpha;
      if (hit) {
        const double q = std_ * std_ + dtd * (dsq - sts);
        const double rad = sqrt(q > 0.0 ? q : 0.0);
        const double den1 = std_ + rad;
        al = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
      }
      double rn = rtr - 2.0 * al * rh + al * al * hh;
      rn = rn > 0.0 ? rn : 0.0;
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
      for (int j = tid; j < d; j += RE_THREADS) {
        const double dj = sD[j];
        sS[j] += al * dj;
        const double r = sR[j] - al * acc[j];
        sR[j] = r;
        if (!hit) sD[j] = r + beta * dj;
      }
      if (hit) break;
      rtr = rn;
      sts = tn;
    }
    // ---- trial point W + step (in the direction slot), trust-region update, acceptance
    double s3[3] = {0.0, 0.0, 0.0};
    for (int j = tid; j < d; j += RE_THREADS) {
      const double sj = sS[j];
      s3[0] += sG[j] * sj;
      s3[1] += sj * sR[j];
      s3[2] += sj * sj;
      sD[j] = sW[j] + sj;
    }
    block_sums<3>(s3, red, parity);
    const double gs = s3[0], pred = -0.5 * (gs - s3[1]), snorm = sqrt(s3[2]);
    double gn2;
    const double fn = value_grad(sD, cur ^ 1, false, gn2);   // trial gradient in acc[0 .. d)
    const double actual = f - fn;
    if (it == 0) delta = fmin(delta, snorm);
    const double den = fn - f - gs;
    const double alr = den <= 0.0 ? sg3 : fmax(sg1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(alr, sg1) * snorm, sg2 * delta);
    else if (actual < eta1 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg2 * delta));
    else if (actual < eta2 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg3 * delta));
    else nd = fmax(delta, fmin(alr * snorm, sg3 * delta));
    delta = nd;
    const bool accept = actual > eta0 * pred;
    const double f_prev = f;
    if (accept) {
      for (int j = tid; j < d; j += RE_THREADS) {
        sW[j] = sD[j];
        sG[j] = acc[j];
      }
      gnorm2 = gn2;
      f = fn;
      cur ^= 1;
      ++it;
      fails = 0;
    } else {
      ++fails;
    }
    const bool not_impr = !accept && fails >= a.max_fail;
    int rc = 0;
    if (accept && sqrt(gnorm2) <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= a.max_iter) rc = 1;
    if (rc > 0) { reason = rc; active = false; }
  }
  __syncthreads();
  for (int j = tid; j < d; j += RE_THREADS) Wg[j] = sW[j];
  if (a.zout != nullptr) {
    const double* zc = Z[cur];
    for (long long i = r0 + tid; i < r1; i += RE_THREADS) a.zout[i] = zc[i];
  }
  if (tid == 0) {
    a.f[e] = f; a.iters[e] = it; a.reason[e] = reason;
    if (a.npass != nullptr) a.npass[e] = npass;
  }
}

// Lean streaming TRON (d_e <= 1024): the same solve as re_tron_csr_kernel with only the GATHERED vector and the
// per-wave accumulators in LDS ((1 + RE_NW) x dmax doubles: 40 KB at dmax 1024, so four workgroups = 16 waves per
// CU instead of two). A thread owns coefficients j = tid + 256 q (q < J) for the whole solve: their CG step and
// residual live in its registers, the gradient at W in global scratch (a.gsc) and W itself is updated in place
// in a.W (both are touched once per TRON iteration by their owner thread only). Held to <= 168 VGPRs (3 waves
// per SIMD): small and mid entities are latency-bound (a pass is a few dependent batches), so more entities in
// flight per CU is more streaming throughput.
// Measured on 43K game5pl-like entities (scripts/re_fused_bench.py, profiles/re_lean_ab_r4.md): 3 waves per SIMD
// (<= 168 VGPRs, 12 waves per CU) with two row groups per batch in function evaluations (one: same total, the 64
// largest entities 33.6 instead of 28.1 ms) and three in Hessian-vector passes (four: +15 %); 4 waves per SIMD
// spills in the row loop (80 ms vs 61 ms for re_tron_csr_kernel)
// waves per lean workgroup (one entity): an A/B switch of the profiling builds (production: RE_NW)
#ifndef LEAN_NW
#define LEAN_NW RE_NW
#endif
#define LEAN_THREADS (LEAN_NW * 64)
// row pass of the lean kernel: quads over padded rows (Q) or the strided row_pass
template <bool Q, int MODE, int LOSS, int U>
__device__ __forceinline__ void lean_pass(const ReTronArgs& a, long long r0, long long r1, const double* vec,
                                          double* acc, const double* Dc, double* Dn, double* Zn, double& fpart) {
  if constexpr (Q) row_pass_q<MODE, LOSS, U, LEAN_NW>(a, r0, r1, vec, acc, Dc, Dn, Zn, fpart);
  else row_pass<MODE, LOSS, U, LEAN_NW>(a, r0, r1, vec, acc, Dc, Dn, Zn, fpart);
}
#ifndef LEAN_WPE
#define LEAN_WPE 3
#endif
#ifndef LEAN_UF
#define LEAN_UF 1
#endif
#ifndef LEAN_UH
#define LEAN_UH 3
#endif
template <int LOSS, int J, bool Q>
__global__ __launch_bounds__(LEAN_THREADS) __attribute__((amdgpu_waves_per_eu(LEAN_WPE, LEAN_WPE)))
void re_tron_lean_kernel(ReTronArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int e = __builtin_amdgcn_readfirstlane(a.order[blockIdx.x]);
  const long long r0 = uniform_i64(a.row_ptr[e]), r1 = uniform_i64(a.row_ptr[e + 1]);
  const long long c0 = uniform_i64(a.col_ptr[e]);
  const int d = (int)(uniform_i64(a.col_ptr[e + 1]) - c0);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int dm = a.dmax;
  double* sD = smem;        // CG direction; W / the trial point during a function evaluation
  double* acc = sD + dm;    // LEAN_NW accumulators; acc[0 .. d) = combined gradient after a function evaluation
  double* red = acc + LEAN_NW * dm;
  double* myacc = acc + w * dm;
  double* D[2] = {a.scr, a.scr + a.n_rows};
  double* Z[2] = {a.scr + 2 * a.n_rows, a.scr + 3 * a.n_rows};
  double* Wg = a.W + c0;
  double* Gg = a.gsc + c0;
  int cur = 0, parity = 0, npass = 0;
  double S[J], R[J];

  auto combined = [&](int j) -> double {
    double g = acc[j];
#pragma unroll
    for (int q = 1; q < LEAN_NW; ++q) g += acc[q * dm + j];
    return g;
  };
  // value + gradient at sD (or at zero); gradient -> acc[0 .. d)
  auto value_grad = [&](bool at_zero, int nb, double& gg) -> double {
    ++npass;
    __syncthreads();
    for (int j = lane; j < d; j += 64) myacc[j] = 0.0;
    double fp = 0.0;
    if (at_zero) lean_pass<Q, 2, LOSS, LEAN_UF>(a, r0, r1, sD, myacc, nullptr, nullptr, nullptr, fp);
    else lean_pass<Q, 1, LOSS, LEAN_UF>(a, r0, r1, sD, myacc, nullptr, D[nb], Z[nb], fp);
    __syncthreads();
    double s3[3] = {fp, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < J; ++q) {
      const int j = tid + LEAN_THREADS * q;
      if (j < d) {
        const double v = at_zero ? 0.0 : sD[j];
        const double g = combined(j) + a.l2 * v;
        acc[j] = g;
        s3[1] += v * v;
        s3[2] += g * g;
      }
    }
    block_sums<3, LEAN_NW>(s3, red, parity);
    gg = s3[2];
    return s3[0] + 0.5 * a.l2 * s3[1];
  };

#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = tid + LEAN_THREADS * q;
    if (j < d) sD[j] = Wg[j];
  }
  double gnorm2;
  double f = value_grad(false, cur, gnorm2);
  double nz[1] = {0.0};
#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = tid + LEAN_THREADS * q;
    if (j < d) {
      Gg[j] = acc[j];
      nz[0] += sD[j] != 0.0 ? 1.0 : 0.0;
    }
  }
  block_sums<1, LEAN_NW>(nz, red, parity);
  double f0z = f, g0n = sqrt(gnorm2);
  bool g0_lazy = false;
  if (nz[0] != 0.0) {
    if (a.xf2 != nullptr) {
      // warm start: the tolerances scale with the zero point's f(0) and ||g(0)|| (Optimizer.scala). f(0) needs only
      // the rows' offsets; ||g(0)|| = ||X_e^T c|| <= ||X_e||_F ||c|| (c_i = w_i l'(o_i)) stands in until a gradient
      // norm comes below the bound's tolerance -- then the exact pass at zero runs (convergence decisions are
      // those of the exact norm). No pass over the entity's entries for the common case.
      double s2[2] = {0.0, 0.0};
      for (long long i = r0 + tid; i < r1; i += LEAN_THREADS) {
        double l, dl, d2;
        loss_t<LOSS>(gld(a.off + i), gld(a.y + i), l, dl, d2);
        const double wi = gld(a.wt + i);
        s2[0] += wi * l;
        s2[1] += (wi * dl) * (wi * dl);
      }
      block_sums<2, LEAN_NW>(s2, red, parity);
      f0z = s2[0];
      g0n = sqrt(gld(a.xf2 + e) * s2[1]) * (1.0 + 1e-6) + 1e-300;
      g0_lazy = true;
    } else {
      double g0;
      f0z = value_grad(true, 0, g0);
      g0n = sqrt(g0);
    }
  }
  const double loss_tol = f0z * a.tol;
  double grad_tol = g0n * a.tol;
  double delta = sqrt(gnorm2);
  int it = 0, fails = 0, reason = 0;
  bool active = true;
  if (delta == 0.0) { reason = 4; active = false; }
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, sg1 = 0.25, sg2 = 0.5, sg3 = 4.0;
  const int guard_max = a.max_iter * (a.max_fail + 1) + 5;
  for (int guard = 0; active && guard < guard_max; ++guard) {
    // truncated CG at W: one Hessian-vector pass, one combine sweep with the five dot products, one update sweep
#pragma unroll
    for (int q = 0; q < J; ++q) {
      const int j = tid + LEAN_THREADS * q;
      const double g = j < d ? Gg[j] : 0.0;
      S[q] = 0.0;
      R[q] = -g;
      if (j < d) sD[j] = -g;
    }
    double rtr = gnorm2, sts = 0.0;
    const double cg_tol2 = 0.01 * gnorm2;        // (0.1 ||g||)^2
    for (int k = 0; k < a.max_cg; ++k) {
      if (!(rtr > cg_tol2)) break;
      ++npass;
      __syncthreads();
      for (int j = lane; j < d; j += 64) myacc[j] = 0.0;
      double fp = 0.0;
      lean_pass<Q, 0, LOSS, LEAN_UH>(a, r0, r1, sD, myacc, D[cur], nullptr, nullptr, fp);
      __syncthreads();
      double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      double H[J];
#pragma unroll
      for (int q = 0; q < J; ++q) {
        const int j = tid + LEAN_THREADS * q;
        H[q] = 0.0;
        if (j < d) {
          const double dj = sD[j];
          const double h = combined(j) + a.l2 * dj;
          H[q] = h;
          s5[0] += dj * h;
          s5[1] += S[q] * dj;
          s5[2] += dj * dj;
          s5[3] += R[q] * h;
          s5[4] += h * h;
        }
      }
      block_sums<5, LEAN_NW>(s5, red, parity);
      const double dhd = s5[0], std_ = s5[1], dtd = s5[2], rh = s5[3], hh = s5[4];
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      double tn = sts + 2.0 * alpha * std_ + alpha * alpha * dtd;
      tn = tn > 0.0 ? tn : 0.0;
      const double dsq = delta * delta;
      const bool hit = tn > dsq;
      double al = alpha;
      if (hit) {
        const double qq = std_ * std_ + dtd * (dsq - sts);
        const double rad = sqrt(qq > 0.0 ? qq : 0.0);
        const double den1 = std_ + rad;
        al = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
      }
      double rn = rtr - 2.0 * al * rh + al * al * hh;
      rn = rn > 0.0 ? rn : 0.0;
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
#pragma unroll
      for (int q = 0; q < J; ++q) {
        const int j = tid + LEAN_THREADS * q;
        if (j < d) {
          const double dj = sD[j];
          S[q] += al * dj;
          const double r = R[q] - al * H[q];
          R[q] = r;
          if (!hit) sD[j] = r + beta * dj;
        }
      }
      if (hit) break;
      rtr = uniform_f64(rn);
      sts = uniform_f64(tn);
    }
    // trial point W + step (in sD), trust-region update, acceptance
    double s3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < J; ++q) {
      const int j = tid + LEAN_THREADS * q;
      if (j < d) {
        const double sj = S[q];
        s3[0] += Gg[j] * sj;
        s3[1] += sj * R[q];
        s3[2] += sj * sj;
        sD[j] = Wg[j] + sj;
      }
    }
    block_sums<3, LEAN_NW>(s3, red, parity);
    const double gs = s3[0], pred = -0.5 * (gs - s3[1]), snorm = sqrt(s3[2]);
    double gn2;
    const double fn = value_grad(false, cur ^ 1, gn2);   // trial gradient in acc[0 .. d)
    const double actual = f - fn;
    if (it == 0) delta = uniform_f64(fmin(delta, snorm));
    const double den = fn - f - gs;
    const double alr = den <= 0.0 ? sg3 : fmax(sg1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(alr, sg1) * snorm, sg2 * delta);
    else if (actual < eta1 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg2 * delta));
    else if (actual < eta2 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg3 * delta));
    else nd = fmax(delta, fmin(alr * snorm, sg3 * delta));
    delta = uniform_f64(nd);
    const bool accept = actual > eta0 * pred;
    const double f_prev = f;
    if (accept) {
#pragma unroll
      for (int q = 0; q < J; ++q) {
        const int j = tid + LEAN_THREADS * q;
        if (j < d) {
          Wg[j] = sD[j];
          Gg[j] = acc[j];
        }
      }
      gnorm2 = gn2;
      f = fn;
      cur ^= 1;
      ++it;
      fails = 0;
    } else {
      ++fails;
    }
    const bool not_impr = !accept && fails >= a.max_fail;
    if (accept && g0_lazy && sqrt(gnorm2) <= grad_tol) {
      // the bound no longer decides: the exact ||g(0)|| (a pass at zero; acc is free, Gg holds the gradient)
      double g0;
      (void)value_grad(true, 0, g0);
      grad_tol = sqrt(g0) * a.tol;
      g0_lazy = false;
    }
    int rc = 0;
    if (accept && sqrt(gnorm2) <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= a.max_iter) rc = 1;
    if (rc > 0) { reason = rc; active = false; }
  }
  __syncthreads();
  if (a.zout != nullptr) {
    const double* zc = Z[cur];
    for (long long i = r0 + tid; i < r1; i += LEAN_THREADS) a.zout[i] = zc[i];
  }
  if (tid == 0) {
    a.f[e] = f; a.iters[e] = it; a.reason[e] = reason;
    if (a.npass != nullptr) a.npass[e] = npass;
  }
}

// ============================================================================================================
// Tall-narrow entities (d_e <= 64 coefficients, typically more rows than coefficients): ONE WAVE PER ENTITY, the
// whole TRON with the EXACT per-entity Hessian H_e = X_e^T D X_e + l2 I. No workgroup barriers: the waves of a
// workgroup are independent entities, every reduction is a DPP / readlane wave sum, LDS hand-offs between the
// lanes of one wave are ordered by wave_sync (in-order LDS per wave + a compiler fence).
// * Coefficient-space vectors live in registers: lane j holds w_j, g_j, step_j, r_j, dir_j (j < d_e <= 64).
// * Row passes stage RT_RB = 16 rows at a time as a dense [16][DP + 4] LDS block (row stride DP + 4: the
//   quad-per-row margin reads are bank-conflict free): the entries are scattered from registers and zeroed again
//   after use, and the NEXT block's entries (and the row pointers two blocks ahead) are already in flight while a
//   block computes, so a pass costs about one global-memory latency, not one per block.
// * Margins: a lane quad per row; gradient: lane j sums X[r][j] t_r over the 16 rows in a fixed order (no
//   atomics: deterministic by construction).
// * Hessian: per 4 staged rows one v_mfma_f64_16x16x4f64 per upper-triangle 16 x 16 tile (all tiles in the one
//   wave, fixed k order), written to LDS EXACTLY symmetric (diagonal tiles mirrored from their upper half), so a
//   CG step reads column j of H (consecutive lanes: conflict-free) for (H d)_j. For d_e <= 32 (FH) the Hessian
//   at the trial point is formed INSIDE the trial point's function evaluation into a second LDS buffer (adopted
//   when the step is accepted): one row pass per TRON iteration. Wider entities run a separate Hessian pass.
// ============================================================================================================
typedef double v4d __attribute__((ext_vector_type(4)));
#define RT_RB 16

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum over the 4 lanes of a quad, in every lane of the quad (fixed order).
__device__ __forceinline__ double quad_total(double v) {
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  return v;
}

template <int T>
struct TallCfg {
  static constexpr int DP = 16 * T;                  // padded coefficient count
  static constexpr int XS = DP + 4;                  // staged row stride (doubles)
  static constexpr bool FH = T <= 2;                 // Hessian fused into the function evaluation (2 H buffers)
  static constexpr int WORDS = (FH ? 2 : 1) * DP * DP + RT_RB * XS + DP + 2 * RT_RB;   // LDS doubles per wave
};

template <int T, int LOSS>
__global__ __launch_bounds__(64) void re_tron_tall_kernel(ReTronArgs a) {
  using C = TallCfg<T>;
  constexpr int DP = C::DP, XS = C::XS, NT = T * (T + 1) / 2, KE = T;
  constexpr bool FH = C::FH;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lane = threadIdx.x;
  const int e = a.order[blockIdx.x];
  double* const H0 = smem;                              // [DP][DP] Hessian buffers, exactly symmetric
  double* const H1 = smem + (FH ? DP * DP : 0);
  double* Xs = smem + (FH ? 2 : 1) * DP * DP;           // [RT_RB][XS] staged rows (zero between blocks)
  double* sV = Xs + RT_RB * XS;                         // [DP] vector broadcast to the lanes (margins / CG)
  double* sT = sV + DP;                                 // [RT_RB] per staged row: gradient weight t_r
  double* sD = sT + RT_RB;                              // [RT_RB] per staged row: Hessian weight D_r
  int hc = 0;                                           // (hc ? H1 : H0) = Hessian at the current point
  const long long r0 = a.row_ptr[e], r1 = a.row_ptr[e + 1];
  const long long c0 = a.col_ptr[e];
  const int d = (int)(a.col_ptr[e + 1] - c0);
  const bool own = lane < d;                            // lane j owns coefficient j
  double* D[2] = {a.scr, a.scr + a.n_rows};
  double* Z[2] = {a.scr + 2 * a.n_rows, a.scr + 3 * a.n_rows};
  int cur = 0, npass = 0;
  double* Wg = a.W + c0;
  const int grp = lane >> 4, gl = lane & 15;
  // entity-local 32-bit offsets from per-entity bases (one VGPR per address)
  const long long e0 = a.nip[r0];
  const uint16_t* __restrict__ lcol = a.lcol + e0;
  const double* __restrict__ val = a.val + e0;
  const int nrows = (int)(r1 - r0);
  for (int i = lane; i < RT_RB * XS; i += 64) Xs[i] = 0.0;

  struct Blk {
    int c[RT_RB / 4][KE];
    double v[RT_RB / 4][KE];
    double rs[3];
  };
  // row pointers of block b (lane q <= RT_RB: entity-local offset of row b + q)
  auto fetch_np = [&](int b) -> int {
    const int ip = b + (lane <= RT_RB ? lane : RT_RB);
    return b < nrows ? (int)(a.nip[r0 + (ip < nrows ? ip : nrows)] - e0) : 0;
  };
  // issue the loads of block b (entries + per-row scalars: mode 0 = D[cur] in rs[0], else wt / off / y)
  auto issue = [&](Blk& B, int b, int np, int mode) {
    B.rs[0] = B.rs[1] = B.rs[2] = 0.0;
    if (lane < RT_RB && b + lane < nrows) {
      const long long i = r0 + b + lane;
      if (mode == 0) B.rs[0] = D[cur][i];
      else { B.rs[0] = a.wt[i]; B.rs[1] = a.off[i]; B.rs[2] = a.y[i]; }
    }
#pragma unroll
    for (int u = 0; u < RT_RB / 4; ++u) {
      const int q = u * 4 + grp;
      const int lo = __shfl(np, q, 64), hi = __shfl(np, q + 1, 64);
#pragma unroll
      for (int k = 0; k < KE; ++k) {
        const int p = lo + gl + 16 * k;
        const bool in = p < hi;
        B.c[u][k] = in ? (int)lcol[p] : -1;
        B.v[u][k] = in ? val[p] : 0.0;
      }
    }
  };
  auto scatter = [&](const Blk& B, bool zero) {
#pragma unroll
    for (int u = 0; u < RT_RB / 4; ++u)
#pragma unroll
      for (int k = 0; k < KE; ++k)
        if (B.c[u][k] >= 0) Xs[(u * 4 + grp) * XS + B.c[u][k]] = zero ? 0.0 : B.v[u][k];
  };
  // Pipelined pass over the entity's blocks: body(b, B) runs with block b staged in Xs (and its loads in B.rs).
  auto pass = [&](int mode, auto&& body) {
    Blk A, B2;
    int np = fetch_np(0);
    issue(A, 0, np, mode);
    np = fetch_np(RT_RB);
    for (int b = 0; b < nrows; b += 2 * RT_RB) {
      const bool hasB = b + RT_RB < nrows;
      if (hasB) issue(B2, b + RT_RB, np, mode);
      np = fetch_np(b + 2 * RT_RB);
      scatter(A, false);
      wave_sync();
      body(b, A);
      wave_sync();
      scatter(A, true);
      if (!hasB) break;
      const bool hasA = b + 2 * RT_RB < nrows;
      if (hasA) issue(A, b + 2 * RT_RB, np, mode);
      np = fetch_np(b + 3 * RT_RB);
      scatter(B2, false);
      wave_sync();
      body(b + RT_RB, B2);
      wave_sync();
      scatter(B2, true);
      if (!hasA) break;
    }
  };
  // MFMA accumulation of X_blk^T diag(w) X_blk for the staged block (w in LDS ``sw``)
  auto hess_block = [&](v4d (&cacc)[NT], const double* sw) {
    const int rr = lane & 15, kk = lane >> 4;
#pragma unroll 1
    for (int kg = 0; kg < RT_RB / 4; ++kg) {
      const int k = kg * 4 + kk;
      const double dk = sw[k];
      const double* xk = Xs + k * XS;
      int t = 0;
#pragma unroll
      for (int ti = 0; ti < T; ++ti)
#pragma unroll
        for (int tj = ti; tj < T; ++tj, ++t)
          cacc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xk[ti * 16 + rr], dk * xk[tj * 16 + rr], cacc[t], 0, 0, 0);
    }
  };
  auto store_hess = [&](v4d (&cacc)[NT], double* H) {
    int t = 0;
#pragma unroll
    for (int ti = 0; ti < T; ++ti)
#pragma unroll
      for (int tj = ti; tj < T; ++tj, ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // accumulator i of lane l holds C[(l >> 4) + 4 i][l & 15] of the tile
          const int lr = (lane >> 4) + 4 * i, lc = lane & 15;
          const int row = ti * 16 + lr, col = tj * 16 + lc;
          if (ti != tj || lr <= lc) {
            H[row * DP + col] = cacc[t][i];
            H[col * DP + row] = cacc[t][i];
          }
        }
    wave_sync();
    if (lane < DP) H[lane * DP + lane] += a.l2;
    wave_sync();
  };

  // value + gradient at the lane-held vector ``vj`` (written to sV here). mode 1: writes Z buffer ``nb`` (and D
  // when the Hessian has its own pass); mode 2 (the state at zero): no scratch writes. ``Hout`` (FH only): the
  // Hessian at vj is formed in the same pass. Returns f; gj = this lane's gradient component (l2 included).
  auto value_grad = [&](double vj, int mode, int nb, double& gj, double* Hout) -> double {
    ++npass;
    if (lane < DP) sV[lane] = own ? vj : 0.0;
    const int r = lane >> 2, q = lane & 3;
    double fp = 0.0, g = 0.0;
    v4d cacc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) cacc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    pass(1, [&](int b, const Blk& B) {
      double s = 0.0;
#pragma unroll 4
      for (int cc = 0; cc < DP / 4; ++cc) s = fma(Xs[r * XS + q + 4 * cc], sV[q + 4 * cc], s);
      s = quad_total(s);
      const double wt = __shfl(B.rs[0], r, 64), of = __shfl(B.rs[1], r, 64), yy = __shfl(B.rs[2], r, 64);
      double t = 0.0, h = 0.0;
      if (b + r < nrows) {
        const long long i = r0 + b + r;
        double l, dl, d2;
        loss_t<LOSS>(s + of, yy, l, dl, d2);
        t = wt * dl;
        h = wt * d2;
        if (q == 0) {
          fp += wt * l;
          if (mode == 1) {
            Z[nb][i] = s;
            if (!FH) D[nb][i] = h;
          }
        }
      }
      if (q == 0) { sT[r] = t; sD[r] = h; }
      wave_sync();
      if (lane < DP) {
#pragma unroll 4
        for (int rr = 0; rr < RT_RB; ++rr) g = fma(Xs[rr * XS + lane], sT[rr], g);
      }
      if (FH && Hout != nullptr) hess_block(cacc, sD);
    });
    if (FH && Hout != nullptr) store_hess(cacc, Hout);
    gj = own ? g + a.l2 * vj : 0.0;
    return wave_total(fp) + 0.5 * a.l2 * wave_total(own ? vj * vj : 0.0);
  };
  // separate Hessian pass at the current point (entities wider than 32): H = X^T diag(D[cur]) X + l2 I
  auto form_hessian = [&]() {
    ++npass;
    v4d cacc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) cacc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    pass(0, [&](int b, const Blk& B) {
      if (lane < RT_RB) sD[lane] = B.rs[0];
      wave_sync();
      hess_block(cacc, sD);
    });
    store_hess(cacc, (hc ? H1 : H0));
  };

  double Wj = own ? Wg[lane] : 0.0, Gj;
  double f = value_grad(Wj, 1, cur, Gj, FH ? (hc ? H1 : H0) : nullptr);
  double gnorm2 = wave_total(Gj * Gj);
  const double nz = wave_total(own && Wj != 0.0 ? 1.0 : 0.0);
  double f0z = f, g0n = sqrt(gnorm2);
  if (nz != 0.0) {
    double g0j;
    f0z = value_grad(0.0, 2, 0, g0j, nullptr);
    g0n = sqrt(wave_total(g0j * g0j));
  }
  const double loss_tol = f0z * a.tol, grad_tol = g0n * a.tol;
  double delta = sqrt(gnorm2);
  int it = 0, fails = 0, reason = 0;
  bool active = true, need_h = !FH;
  if (delta == 0.0) { reason = 4; active = false; }
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, sg1 = 0.25, sg2 = 0.5, sg3 = 4.0;
  const int guard_max = a.max_iter * (a.max_fail + 1) + 5;
  for (int guard = 0; active && guard < guard_max; ++guard) {
    if (need_h) { form_hessian(); need_h = false; }
    const double* H = (hc ? H1 : H0);
    // ---- truncated CG on the LDS Hessian: per step one column-read mat-vec and five wave sums
    double Sj = 0.0, Rj = -Gj, Dj = -Gj;
    double rtr = gnorm2, sts = 0.0;
    const double cg_tol2 = 0.01 * gnorm2;
    for (int k = 0; k < a.max_cg; ++k) {
      if (!(rtr > cg_tol2)) break;
      if (lane < DP) sV[lane] = Dj;
      wave_sync();
      double h0 = 0.0, h1 = 0.0;
      if (lane < DP) {
#pragma unroll 2
        for (int cc = 0; cc < DP; cc += 2) {
          h0 = fma(H[cc * DP + lane], sV[cc], h0);
          h1 = fma(H[(cc + 1) * DP + lane], sV[cc + 1], h1);
        }
      }
      wave_sync();
      const double hj = own ? h0 + h1 : 0.0;
      const double dhd = wave_total(Dj * hj), std_ = wave_total(Sj * Dj), dtd = wave_total(Dj * Dj);
      const double rh = wave_total(Rj * hj), hh = wave_total(hj * hj);
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      double tn = sts + 2.0 * alpha * std_ + alpha * alpha * dtd;
      tn = tn > 0.0 ? tn : 0.0;
      const double dsq = delta * delta;
      const bool hit = tn > dsq;
      double al = alpha;
      if (hit) {
        const double qq = std_ * std_ + dtd * (dsq - sts);
        const double rad = sqrt(qq > 0.0 ? qq : 0.0);
        const double den1 = std_ + rad;
        al = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
      }
      double rn = rtr - 2.0 * al * rh + al * al * hh;
      rn = rn > 0.0 ? rn : 0.0;
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
      Sj += al * Dj;
      Rj -= al * hj;
      if (hit) break;
      Dj = Rj + beta * Dj;
      rtr = rn;
      sts = tn;
    }
    // ---- trial point (its Hessian formed in the same pass when FH), trust-region update, acceptance
    const double gs = wave_total(Gj * Sj), pred = -0.5 * (gs - wave_total(Sj * Rj)), snorm = sqrt(wave_total(Sj * Sj));
    const double Tj = own ? Wj + Sj : 0.0;
    double Gn;
    const double fn = value_grad(Tj, 1, cur ^ 1, Gn, FH ? (hc ? H0 : H1) : nullptr);
    const double gn2 = wave_total(Gn * Gn);
    const double actual = f - fn;
    if (it == 0) delta = fmin(delta, snorm);
    const double den = fn - f - gs;
    const double alr = den <= 0.0 ? sg3 : fmax(sg1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(alr, sg1) * snorm, sg2 * delta);
    else if (actual < eta1 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg2 * delta));
    else if (actual < eta2 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg3 * delta));
    else nd = fmax(delta, fmin(alr * snorm, sg3 * delta));
    delta = nd;
    const bool accept = actual > eta0 * pred;
    const double f_prev = f;
    if (accept) {
      Wj = Tj;
      Gj = Gn;
      gnorm2 = gn2;
      f = fn;
      cur ^= 1;
      ++it;
      fails = 0;
      if (FH) hc ^= 1;
      else need_h = true;
    } else {
      ++fails;
    }
    const bool not_impr = !accept && fails >= a.max_fail;
    int rc = 0;
    if (accept && sqrt(gnorm2) <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= a.max_iter) rc = 1;
    if (rc > 0) { reason = rc; active = false; }
  }
  if (own) Wg[lane] = Wj;
  if (a.zout != nullptr) {
    const double* zc = Z[cur];
    for (long long i = r0 + lane; i < r1; i += 64) a.zout[i] = zc[i];
  }
  if (lane == 0) {
    a.f[e] = f; a.iters[e] = it; a.reason[e] = reason;
    if (a.npass != nullptr) a.npass[e] = npass;
  }
}

// ============================================================================================================
// Row-space TRON for WIDE entities of 64 < n_e <= 192 rows (optimization/row_space.py: the entity's problem is the
// dense GLM with the n x n lower-triangular design matrix L_e, K_e = X_e X_e^T = L_e L_e^T). The n <= 64 classes
// run rs_tron_kernel / rs_tron_dpp_kernel (glm_kernels.hip); here ONE WAVE owns one problem with E = ceil(n / 64)
// vector entries per lane (lane l: entries l, l + 64, ...), L's packed lower triangle is staged once into the
// wave's LDS, every sum is a DPP / readlane wave sum (no workgroup barriers) and the whole TRON runs in the kernel.
// Against the primal fused kernel on such an entity (d_e ~ 1000 coefficients, ~50 non-zeros per row) every CG
// step is two LDS-resident triangular mat-vecs over n-length vectors instead of a pass over the rows' non-zeros
// plus d-length vector work. Same TRON semantics as rs_tron_kernel (photon-lib/.../optimization/TRON.scala).
// ============================================================================================================
template <int E, int LOSS>
__global__ __launch_bounds__(64) void rs_tron_big_kernel(int B, int n, const double* __restrict__ Lm,
                                                         const double* __restrict__ Y, const double* __restrict__ O,
                                                         const double* __restrict__ WT, double* __restrict__ Beta,
                                                         double* __restrict__ Fout, int* __restrict__ Iters,
                                                         int* __restrict__ Reason, double* __restrict__ Zout,
                                                         double l2, double tol, int max_iter, int max_fail,
                                                         int max_cg) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lane = threadIdx.x;
  const long long b = blockIdx.x;
  if (b >= B) return;
  const int np = n * (n + 1) / 2;
  double* Lp = smem;              // packed lower triangle: L[r][c] (c <= r) at r (r + 1) / 2 + c
  double* sv = smem + np;         // [n] vector broadcast to the lanes
  const double* Lb = Lm + b * (long long)n * n;
  for (int r = 0; r < n; ++r)
    for (int c = lane; c <= r; c += 64) Lp[r * (r + 1) / 2 + c] = Lb[(long long)r * n + c];
  bool on[E];
  double y[E], off[E], wt[E], W[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane + 64 * e;
    on[e] = i < n;
    const long long o = b * n + (on[e] ? i : 0);
    y[e] = on[e] ? Y[o] : 0.0;
    off[e] = on[e] ? O[o] : 0.0;
    wt[e] = on[e] ? WT[o] : 0.0;
    W[e] = on[e] ? Beta[o] : 0.0;
  }
  wave_sync();
  auto gsum = [&](const double (&v)[E]) -> double {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) s += v[e];
    return wave_total(s);
  };
  auto gsum2 = [&](const double (&u)[E], const double (&v)[E]) -> double {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) s = fma(u[e], v[e], s);
    return wave_total(s);
  };
  auto put = [&](const double (&v)[E]) {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (on[e]) sv[lane + 64 * e] = v[e];
    wave_sync();
  };
  auto mv = [&](const double (&v)[E], double (&out)[E]) {     // (L v)_i
    put(v);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = on[e] ? lane + 64 * e : 0;
      const double* Lr = Lp + i * (i + 1) / 2;
      double a0 = 0.0, a1 = 0.0;
      int j = 0;
      for (; j + 1 <= i; j += 2) {
        a0 = fma(Lr[j], sv[j], a0);
        a1 = fma(Lr[j + 1], sv[j + 1], a1);
      }
      if (j <= i) a0 = fma(Lr[j], sv[j], a0);
      out[e] = on[e] ? a0 + a1 : 0.0;
    }
    wave_sync();                       // sv reads done before the next put
  };
  auto mvt = [&](const double (&u)[E], double (&out)[E]) {    // (L^T u)_i
    put(u);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = on[e] ? lane + 64 * e : 0;
      double a0 = 0.0, a1 = 0.0;
      int r = i;
      for (; r + 1 < n; r += 2) {
        a0 = fma(Lp[r * (r + 1) / 2 + i], sv[r], a0);
        a1 = fma(Lp[(r + 1) * (r + 2) / 2 + i], sv[r + 1], a1);
      }
      if (r < n) a0 = fma(Lp[r * (r + 1) / 2 + i], sv[r], a0);
      out[e] = on[e] ? a0 + a1 : 0.0;
    }
    wave_sync();
  };
  // value, gradient and Hessian weights at v; z (margins L v, no offset) kept for the output
  auto vg = [&](const double (&v)[E], double& f, double (&gr)[E], double (&Dw)[E], double (&z)[E]) {
    mv(v, z);
    double t[E], fl[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      double l = 0.0, dl = 0.0, d2 = 0.0;
      if (on[e]) loss_t<LOSS>(z[e] + off[e], y[e], l, dl, d2);
      fl[e] = wt[e] * l + 0.5 * l2 * v[e] * v[e];
      t[e] = wt[e] * dl;
      Dw[e] = wt[e] * d2;
    }
    f = gsum(fl);
    mvt(t, gr);
#pragma unroll
    for (int e = 0; e < E; ++e) gr[e] = on[e] ? gr[e] + l2 * v[e] : 0.0;
  };
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, s1 = 0.25, s2 = 0.5, s3 = 4.0;
  double f, gr[E], Dw[E], Z[E];
  vg(W, f, gr, Dw, Z);
  double f0z, g0n;
  double nzv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) nzv[e] = W[e] != 0.0 ? 1.0 : 0.0;
  if (gsum(nzv) == 0.0) {
    f0z = f;
    g0n = sqrt(gsum2(gr, gr));
  } else {
    double zero[E], g0[E], D0[E], z0[E];
#pragma unroll
    for (int e = 0; e < E; ++e) zero[e] = 0.0;
    vg(zero, f0z, g0, D0, z0);
    g0n = sqrt(gsum2(g0, g0));
  }
  const double loss_tol = f0z * tol, grad_tol = g0n * tol;
  double delta = sqrt(gsum2(gr, gr));
  int it = 0, fails = 0, reason = 0;
  bool active = true;
  if (delta == 0.0) { reason = 4; active = false; }
  const int guard_max = max_iter * (max_fail + 1) + 5;
  for (int guard = 0; active && guard < guard_max; ++guard) {
    // ---- truncated CG at W (Hessian weights Dw of the current iterate)
    double step[E], r[E], d[E];
#pragma unroll
    for (int e = 0; e < E; ++e) { step[e] = 0.0; r[e] = -gr[e]; d[e] = r[e]; }
    double rtr = gsum2(r, r);
    const double cg_tol = 0.1 * sqrt(gsum2(gr, gr));
    for (int k = 0; k < max_cg; ++k) {
      if (!(sqrt(rtr > 0.0 ? rtr : 0.0) > cg_tol)) break;
      double Ld[E], Hd[E], Hl[E];
      mv(d, Ld);
#pragma unroll
      for (int e = 0; e < E; ++e) Ld[e] *= Dw[e];
      mvt(Ld, Hd);
#pragma unroll
      for (int e = 0; e < E; ++e) Hl[e] = Hd[e] + l2 * d[e];
      const double dhd = gsum2(d, Hl), std_ = gsum2(step, d), sts = gsum2(step, step), dtd = gsum2(d, d);
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      double tr[E];
#pragma unroll
      for (int e = 0; e < E; ++e) tr[e] = step[e] + alpha * d[e];
      const double tn = gsum2(tr, tr);
      const bool hit = sqrt(tn > 0.0 ? tn : 0.0) > delta;
      double a = alpha;
      if (hit) {
        const double dsq = delta * delta;
        const double q = std_ * std_ + dtd * (dsq - sts);
        const double rad = sqrt(q > 0.0 ? q : 0.0);
        const double den1 = std_ + rad;
        a = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
      }
      double rn_v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        step[e] = step[e] + a * d[e];
        rn_v[e] = r[e] - a * Hl[e];
      }
      const double rn = gsum2(rn_v, rn_v);
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        r[e] = rn_v[e];
        if (!hit) d[e] = rn_v[e] + beta * d[e];
      }
      if (hit) break;
      rtr = rn;
    }
    // ---- trial point, trust-region update, acceptance
    double Wn[E];
#pragma unroll
    for (int e = 0; e < E; ++e) Wn[e] = W[e] + step[e];
    const double gs = gsum2(gr, step);
    const double pred = -0.5 * (gs - gsum2(step, r));
    double fn, gn[E], Dn[E], Zn[E];
    vg(Wn, fn, gn, Dn, Zn);
    const double actual = f - fn;
    const double snorm = sqrt(gsum2(step, step));
    if (it == 0) delta = fmin(delta, snorm);
    const double den = fn - f - gs;
    const double al = den <= 0.0 ? s3 : fmax(s1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(al, s1) * snorm, s2 * delta);
    else if (actual < eta1 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s2 * delta));
    else if (actual < eta2 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s3 * delta));
    else nd = fmax(delta, fmin(al * snorm, s3 * delta));
    delta = nd;
    const bool accept = actual > eta0 * pred;
    const double f_prev = f;
    if (accept) {
#pragma unroll
      for (int e = 0; e < E; ++e) { W[e] = Wn[e]; gr[e] = gn[e]; Dw[e] = Dn[e]; Z[e] = Zn[e]; }
      f = fn;
      ++it;
      fails = 0;
    } else {
      ++fails;
    }
    const bool not_impr = !accept && fails >= max_fail;
    const double gnorm = sqrt(gsum2(gr, gr));
    int rc = 0;
    if (accept && gnorm <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= max_iter) rc = 1;
    if (rc > 0) { reason = rc; active = false; }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (!on[e]) continue;
    const long long o = b * n + lane + 64 * e;
    Beta[o] = W[e];
    if (Zout != nullptr) Zout[o] = Z[e];
  }
  if (lane == 0) { Fout[b] = f; Iters[b] = it; Reason[b] = reason; }
}

// ============================================================================================================
// REGISTER-RESIDENT fused primal TRON (wide entities: d_e <= 1024, rows of <= 64 non-zeros).
// The fused kernel above streams an entity's CSR rows from memory for every Hessian-vector product (~36 row
// passes per solve at ~3.6 TB/s). Here the rows are loaded ONCE into VGPRs and every later pass runs on-chip:
// * a workgroup of RS_NW = 8 waves holds up to RS_CAP = 8 x 4 x S rows: row r -> slot group sg = r / 4, wave
//   sg % 8, register slot sg / 8; 16 lanes per row, lane k of the row keeps entries k, k + 16, k + 32, k + 48
//   (fp64 value + packed u16 column). Per-row D (current / trial), margins (current / trial), weight, offset and
//   label sit in LDS; the coefficient vectors and one accumulator per wave in LDS as in the streaming kernel.
// * entities longer than RS_CAP rows are split over a CLUSTER of k workgroups (member m holds rows
//   [m RS_CAP, (m + 1) RS_CAP)): after every row pass each member publishes its partial sum (d doubles + the
//   loss), the members meet at a cluster barrier (agent-scope release / acquire on a per-task counter), and
//   every member sums the k partials in member order. All control flow then derives from identical sums, so the
//   k replicas of the TRON state stay bitwise identical and no other exchange is needed.
// * ONE persistent launch (one workgroup per CU, grid = resident capacity) serves every task: a workgroup
//   dequeues a ticket (one atomic), a task with k members owns k consecutive tickets (largest tasks first).
//   Tickets are taken in order by running workgroups only, so the earliest incomplete cluster is always filled
//   by workgroups finishing earlier tasks: deadlock-free while k <= the resident workgroups. Every wait is
//   bounded anyway (~1 s, then a global error flag releases every waiter and the host raises).
// Deterministic: fixed-order DPP row sums, per-wave LDS accumulators combined in wave order, member partials
// combined in member order (same LDS ds_add_f64 lane-order assumption as the streaming kernel inside a wave).
// ============================================================================================================
#define RS_NW 8
#define RS_THREADS (RS_NW * 64)
#define RS_DMAX 1024
#define RES_S 12              // register slots per wave (rows per workgroup = 8 x 4 x RES_S)

template <int K>
__device__ __forceinline__ void block_sums8(double (&v)[K], double* __restrict__ red, int& parity) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_total(v[k]);
  double* slot = red + parity * (RS_NW * 8);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) slot[w * 8 + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < RS_NW; ++q) s += slot[q * 8 + k];
    v[k] = s;
    __builtin_amdgcn_sched_barrier(0);    // one value at a time (8 LDS reads), not 8 x K reads in flight
  }
  parity ^= 1;
}

struct ResTasks {
  int* ticket;               // dequeue counter (zero before the launch)
  const int* task_ent;       // [n_tasks] entity
  const int* task_t0;        // [n_tasks + 1] first ticket of each task (task j has task_t0[j+1] - task_t0[j] members)
  int n_tasks;
  unsigned* bar;             // [n_tasks] cluster barrier counters (zero before the launch)
  double* ws;                // [n_tickets][2][RS_DMAX + 8] member partials (double-buffered by pass parity)
  int* err;                  // set when a cluster wait timed out (the results are then invalid)
};

// Cluster barrier of the k members of one task (k > 1). Producer: every wave drains its stores, workgroup barrier,
// one lane releases at agent scope and adds to the task's counter; consumer: relaxed polls of the counter, one
// agent-scope acquire, workgroup barrier (MI355X_MICROARCH.md, valid hand-off forms). Bounded: ~1 s, then err.
__device__ __forceinline__ void cluster_barrier(unsigned* bar, unsigned target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {      // 1 s at the 100 MHz constant clock
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int S, int LOSS>
__global__ __launch_bounds__(RS_THREADS) void re_tron_res_kernel(ReTronArgs a, ResTasks tk) {
  constexpr int CAP = RS_NW * 4 * S;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int grp = lane >> 4, gl = lane & 15;
  constexpr int DM = RS_DMAX, DMS = RS_DMAX + 8;   // + a dummy slot (index DM) for the empty register entries
  double* sV = smem;                  // [DMS] gathered vector: CG direction / trial point (sV[DM] == 0)
  double* sH = sV + DMS;              // combined Hessian-vector product / trial gradient
  double* sW = sH + DM;
  double* sG = sW + DM;
  double* sS = sG + DM;              // CG step
  double* sR = sS + DM;              // CG residual
  double* acc = sR + DM;             // [RS_NW][DMS] per-wave accumulators (zero between passes)
  double* rD = acc + RS_NW * DMS;    // [2][CAP] per local row: Hessian weight D (current / trial)
  double* rZ = rD + 2 * CAP;         // [2][CAP] margins x.w (current / trial)
  double* rW = rZ + 2 * CAP;         // [CAP] weight
  double* rO = rW + CAP;             // [CAP] offset
  double* rY = rO + CAP;             // [CAP] label
  double* red = rY + CAP;            // [2][RS_NW][8], then [16] TRON scalars
  double* myacc = acc + w * DMS;
  __shared__ int sTicket;
  for (int i = tid; i < RS_NW * DMS; i += RS_THREADS) acc[i] = 0.0;
  if (tid < 8) sV[DM + tid] = 0.0;

  for (;;) {
    __syncthreads();
    if (tid == 0) sTicket = atomicAdd(tk.ticket, 1);
    __syncthreads();
    const int t = sTicket;
    if (t >= tk.task_t0[tk.n_tasks]) break;
    // task of ticket t: the last j with task_t0[j] <= t
    int lo = 0, hi = tk.n_tasks - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tk.task_t0[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int j = lo, m = t - tk.task_t0[j], k = tk.task_t0[j + 1] - tk.task_t0[j];
    const int e = tk.task_ent[j];
    unsigned* bar = tk.bar + j;
    unsigned epoch = 0;
    double* wsm = tk.ws + (size_t)tk.task_t0[j] * 2 * (DM + 8);   // member 0's partials; member q at + q * 2 (DM + 8)
    const long long r0 = a.row_ptr[e];
    const long long rb = r0 + (long long)m * CAP;                  // this member's first row
    const int nloc = (int)min((long long)CAP, a.row_ptr[e + 1] - rb);
    const long long c0 = a.col_ptr[e];
    const int d = (int)(a.col_ptr[e + 1] - c0);
    int cur = 0, parity = 0, npass = 0, wpar = 0;
    double* Wg = a.W + c0;

    // ---- load this member's rows into registers, its row scalars into LDS
    double xv[S][4];
    uint32_t xc[S][2];
    // number of register slots of this wave holding rows: sg = s * RS_NW + w < ceil(nloc / 4)
    const int nsg = (nloc + 3) >> 2;
    const int ns = nsg > w ? (nsg - w + RS_NW - 1) / RS_NW : 0;
    {
      // member-local 32-bit entry offsets (one VGPR per address); loads issued 4 slots at a time
      const long long eb = a.nip[rb];
      const uint16_t* __restrict__ lc = a.lcol + eb;
      const double* __restrict__ vl = a.val + eb;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int r = ((s * RS_NW + w) << 2) + grp;
        int p0 = 0, p1 = 0;
        if (s < ns && r < nloc) { p0 = (int)(a.nip[rb + r] - eb); p1 = (int)(a.nip[rb + r + 1] - eb); }
        uint32_t cc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = p0 + gl + 16 * q;
          const bool in = p < p1;
          xv[s][q] = in ? vl[p] : 0.0;
          cc[q] = in ? (uint32_t)lc[p] : (uint32_t)DM;
        }
        xc[s][0] = cc[0] | (cc[1] << 16);
        xc[s][1] = cc[2] | (cc[3] << 16);
        if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
    }
    for (int r = tid; r < nloc; r += RS_THREADS) {
      rW[r] = a.wt[rb + r];
      rO[r] = a.off[rb + r];
      rY[r] = a.y[rb + r];
    }
    for (int jj = tid; jj < d; jj += RS_THREADS) sW[jj] = Wg[jj];

    // One pass over the resident rows. MODE 0: myacc += X^T (D_cur * (X sV)); MODE 1: value + gradient at sV
    // (myacc += X^T (w l'), fpart, trial D / margins -> rD / rZ slot nb); MODE 2: value + gradient at zero.
    auto pass = [&](int mode, int nb, double& fpart) __attribute__((always_inline)) {
      const double* Dc = rD + cur * CAP;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s < ns) {
          int r = ((s * RS_NW + w) << 2) + grp;
          uint32_t p0 = xc[s][0], p1 = xc[s][1];
          // opaque per pass: keeps the compiler from hoisting the decoded LDS addresses of every entry and row
          // out of the solve loops (that doubled the registers of the resident rows)
          asm volatile("" : "+v"(p0), "+v"(p1), "+v"(r));
          const bool valid = r < nloc;
          const uint32_t c[4] = {p0 & 0xFFFFu, p0 >> 16, p1 & 0xFFFFu, p1 >> 16};
          double dot = 0.0;
          if (mode != 2) {
#pragma unroll
            for (int q = 0; q < 4; ++q) dot = fma(xv[s][q], sV[c[q]], dot);
            dot = row16_total(dot);
          }
          double tt = 0.0;
          if (valid) {
            if (mode == 0) {
              tt = Dc[r] * dot;
            } else {
              const double wt = rW[r];
              double l, dl, d2;
              loss_t<LOSS>(dot + rO[r], rY[r], l, dl, d2);
              tt = wt * dl;
              if (gl == 0) {
                fpart += wt * l;
                if (mode == 1) { rD[nb * CAP + r] = wt * d2; rZ[nb * CAP + r] = dot; }
              }
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) atomicAdd(&myacc[c[q]], tt * xv[s][q]);
        }
        __builtin_amdgcn_sched_barrier(0);   // one slot at a time: no hoisting of later slots' gathers
      }
    };
    // Combine the wave accumulators of this member (and zero them), then the members' partials: out[jj] =
    // sum, for jj < d, in every member identically. ``fp`` (this workgroup's loss part, already block-summed)
    // is combined the same way and returned.
    auto combine = [&](double* out, double fp) __attribute__((always_inline)) -> double {
      __syncthreads();
      if (k == 1) {
        for (int jj = tid; jj < d; jj += RS_THREADS) {
          double h = 0.0;
#pragma unroll
          for (int q = 0; q < RS_NW; ++q) { h += acc[q * DMS + jj]; acc[q * DMS + jj] = 0.0; }
          out[jj] = h;
        }
        __syncthreads();
        return fp;
      }
      double* mine = wsm + (size_t)(m * 2 + wpar) * (DM + 8);
      for (int jj = tid; jj < d; jj += RS_THREADS) {
        double h = 0.0;
#pragma unroll
        for (int q = 0; q < RS_NW; ++q) { h += acc[q * DMS + jj]; acc[q * DMS + jj] = 0.0; }
        mine[jj] = h;
      }
      if (tid == 0) mine[DM] = fp;
      ++epoch;
      cluster_barrier(bar, epoch * (unsigned)k, tk.err);
      for (int jj = tid; jj < d; jj += RS_THREADS) {
        double h = 0.0;
        for (int q = 0; q < k; ++q) h += wsm[(size_t)(q * 2 + wpar) * (DM + 8) + jj];
        out[jj] = h;
      }
      double f = 0.0;
      for (int q = 0; q < k; ++q) f += wsm[(size_t)(q * 2 + wpar) * (DM + 8) + DM];
      wpar ^= 1;
      __syncthreads();
      return f;
    };
    // value + gradient at vec (LDS, written to sV first): gradient (l2 included) -> sH; returns f, gg = ||g||^2.
    auto value_grad = [&](const double* vec, int mode, int nb, double& gg) __attribute__((always_inline)) -> double {
      ++npass;
      __syncthreads();
      if (vec != sV)
        for (int jj = tid; jj < d; jj += RS_THREADS) sV[jj] = mode == 2 ? 0.0 : vec[jj];
      __syncthreads();
      double fp[1] = {0.0};
      pass(mode, nb, fp[0]);
      block_sums8<1>(fp, red, parity);
      const double f = combine(sH, fp[0]);
      double s2[2] = {0.0, 0.0};
      for (int jj = tid; jj < d; jj += RS_THREADS) {
        const double v = sV[jj];
        const double g = sH[jj] + a.l2 * v;
        sH[jj] = g;
        s2[0] += v * v;
        s2[1] += g * g;
      }
      block_sums8<2>(s2, red, parity);
      gg = s2[1];
      return f + 0.5 * a.l2 * s2[0];
    };

    // The TRON scalars live in LDS (every thread writes the same value, so no extra barriers): across the row
    // passes nothing but the resident rows and a few indices stays in VGPRs (no spills into the pass loop).
    double* T = red + 2 * RS_NW * 8;      // [16] scalar state
    int* TI = (int*)(T + 12);             // it, fails, reason, active
    enum { F = 0, GN2 = 1, DELTA = 2, LTOL = 3, GTOL = 4, RTR = 5, STS = 6, CGTOL = 7 };
    {
      double gnorm2;
      const double f = value_grad(sW, 1, cur, gnorm2);
      T[F] = f;
      T[GN2] = gnorm2;
    }
    double nz[1] = {0.0};
    for (int jj = tid; jj < d; jj += RS_THREADS) {
      sG[jj] = sH[jj];
      nz[0] += sW[jj] != 0.0 ? 1.0 : 0.0;
    }
    block_sums8<1>(nz, red, parity);
    {
      double f0z = T[F], g0n = sqrt(T[GN2]);
      if (nz[0] != 0.0) {
        double g0;
        f0z = value_grad(sS, 2, 0, g0);
        g0n = sqrt(g0);
      }
      T[LTOL] = f0z * a.tol;
      T[GTOL] = g0n * a.tol;
      T[DELTA] = sqrt(T[GN2]);
      TI[0] = 0; TI[1] = 0; TI[2] = T[DELTA] == 0.0 ? 4 : 0; TI[3] = T[DELTA] == 0.0 ? 0 : 1;
    }
    const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, sg1 = 0.25, sg2 = 0.5, sg3 = 4.0;
    const int guard_max = a.max_iter * (a.max_fail + 1) + 5;
    for (int guard = 0; TI[3] && guard < guard_max; ++guard) {
      for (int jj = tid; jj < d; jj += RS_THREADS) {
        sS[jj] = 0.0;
        sR[jj] = -sG[jj];
        sV[jj] = -sG[jj];
      }
      T[RTR] = T[GN2];
      T[STS] = 0.0;
      T[CGTOL] = 0.01 * T[GN2];
      for (int kk = 0; kk < a.max_cg; ++kk) {
        // state read BEFORE this step's barriers: a faster thread overwrites RTR / STS after the block sum
        const double rtr = T[RTR], sts = T[STS], delta = T[DELTA];
        if (!(rtr > T[CGTOL])) break;
        ++npass;
        __syncthreads();
        double fpz = 0.0;
        pass(0, 0, fpz);
        combine(sH, 0.0);
        double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int jj = tid; jj < d; jj += RS_THREADS) {
          const double dj = sV[jj];
          const double h = sH[jj] + a.l2 * dj;
          sH[jj] = h;
          s5[0] += dj * h;
          s5[1] += sS[jj] * dj;
          s5[2] += dj * dj;
          s5[3] += sR[jj] * h;
          s5[4] += h * h;
        }
        block_sums8<5>(s5, red, parity);
        const double dhd = s5[0], std_ = s5[1], dtd = s5[2], rh = s5[3], hh = s5[4];
        const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
        double tn = sts + 2.0 * alpha * std_ + alpha * alpha * dtd;
        tn = tn > 0.0 ? tn : 0.0;
        const double dsq = delta * delta;
        const bool hit = tn > dsq;
        double al = alpha;
        if (hit) {
          const double qq = std_ * std_ + dtd * (dsq - sts);
          const double rad = sqrt(qq > 0.0 ? qq : 0.0);
          const double den1 = std_ + rad;
          al = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
        }
        double rn = rtr - 2.0 * al * rh + al * al * hh;
        rn = rn > 0.0 ? rn : 0.0;
        const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
        for (int jj = tid; jj < d; jj += RS_THREADS) {
          const double dj = sV[jj];
          sS[jj] += al * dj;
          const double r = sR[jj] - al * sH[jj];
          sR[jj] = r;
          if (!hit) sV[jj] = r + beta * dj;
        }
        if (hit) break;
        T[RTR] = rn;
        T[STS] = tn;
      }
      // ---- trial point W + step (into sV), trust-region update, acceptance
      __syncthreads();
      double s3[3] = {0.0, 0.0, 0.0};
      for (int jj = tid; jj < d; jj += RS_THREADS) {
        const double sj = sS[jj];
        s3[0] += sG[jj] * sj;
        s3[1] += sj * sR[jj];
        s3[2] += sj * sj;
        sV[jj] = sW[jj] + sj;
      }
      block_sums8<3>(s3, red, parity);
      const double gs = s3[0], pred = -0.5 * (gs - s3[1]), snorm = sqrt(s3[2]);
      // state read BEFORE the trial evaluation's barriers (a faster thread rewrites it after them)
      const double f = T[F], gn2_old = T[GN2];
      double delta = T[DELTA];
      int it = TI[0], fails = TI[1];
      double gn2;
      const double fn = value_grad(sV, 1, cur ^ 1, gn2);     // trial gradient in sH
      const double actual = f - fn;
      if (it == 0) delta = fmin(delta, snorm);
      const double den = fn - f - gs;
      const double alr = den <= 0.0 ? sg3 : fmax(sg1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
      double nd;
      if (actual < eta0 * pred) nd = fmin(fmax(alr, sg1) * snorm, sg2 * delta);
      else if (actual < eta1 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg2 * delta));
      else if (actual < eta2 * pred) nd = fmax(sg1 * delta, fmin(alr * snorm, sg3 * delta));
      else nd = fmax(delta, fmin(alr * snorm, sg3 * delta));
      T[DELTA] = nd;
      const bool accept = actual > eta0 * pred;
      double fc = f, gnc = gn2_old;
      if (accept) {
        for (int jj = tid; jj < d; jj += RS_THREADS) {
          sW[jj] = sV[jj];
          sG[jj] = sH[jj];
        }
        gnc = gn2;
        fc = fn;
        cur ^= 1;
        ++it;
        fails = 0;
      } else {
        ++fails;
      }
      T[GN2] = gnc;
      T[F] = fc;
      const bool not_impr = !accept && fails >= a.max_fail;
      int rc = 0;
      if (accept && sqrt(gnc) <= T[GTOL]) rc = 4;
      if (accept && fabs(fc - f) <= T[LTOL]) rc = 3;
      if (not_impr) rc = 2;
      if ((accept || not_impr) && it >= a.max_iter) rc = 1;
      TI[0] = it;
      TI[1] = fails;
      if (rc > 0) { TI[2] = rc; TI[3] = 0; }
    }
    __syncthreads();
    if (m == 0)
      for (int jj = tid; jj < d; jj += RS_THREADS) Wg[jj] = sW[jj];
    if (a.zout != nullptr)
      for (int r = tid; r < nloc; r += RS_THREADS) a.zout[rb + r] = rZ[cur * CAP + r];
    if (tid == 0 && m == 0) {
      a.f[e] = T[F]; a.iters[e] = TI[0]; a.reason[e] = TI[2];
      if (a.npass != nullptr) a.npass[e] = npass;
    }
  }
}

template <int LOSS, bool Q>
static void lean_launch(const ReTronArgs& a, int n_launch, size_t smem, hipStream_t st) {
  // J coefficients per thread: the smallest of 1 / 2 / 4 with J x LEAN_THREADS >= dmax (dmax <= 1024)
  if (a.dmax <= LEAN_THREADS)
    hipLaunchKernelGGL((re_tron_lean_kernel<LOSS, 1, Q>), dim3(n_launch), dim3(LEAN_THREADS), smem, st, a);
  else if (a.dmax <= 2 * LEAN_THREADS)
    hipLaunchKernelGGL((re_tron_lean_kernel<LOSS, 2, Q>), dim3(n_launch), dim3(LEAN_THREADS), smem, st, a);
  else hipLaunchKernelGGL((re_tron_lean_kernel<LOSS, 4, Q>), dim3(n_launch), dim3(LEAN_THREADS), smem, st, a);
}

extern "C" {

const char* pml_build_id() { return pml_build_stamp + 13; }

// Shared memory of one workgroup for entities of at most ``dmax`` coefficients.
size_t pml_re_tron_smem(int dmax) { return ((size_t)(5 + RE_NW) * dmax + 2 * RE_NW * 8) * sizeof(double); }

int pml_re_tron_csr(const int* order, int n_launch, const long long* row_ptr, const long long* col_ptr,
                    const long long* nip, const uint16_t* lcol, const double* val, const double* y,
                    const double* off, const double* wt, double* scr, long long n_rows, double* W, double* f,
                    int* iters, int* reason, double* zout, int* npass, int loss, double l2, double tol,
                    int max_iter, int max_fail, int max_cg, int dmax, hipStream_t st) {
  if (n_launch <= 0) return 0;
  if (dmax <= 0 || loss < 0 || loss > 2) return -22;
  const size_t smem = pml_re_tron_smem(dmax);
  if (smem > 160 * 1024) return -22;
  ReTronArgs a{order, n_launch, row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr, n_rows, W, f, iters, reason,
               zout, npass, loss, l2, tol, max_iter, max_fail, max_cg, dmax};
  if (loss == LOSS_LOGISTIC) hipLaunchKernelGGL(re_tron_csr_kernel<0>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  else if (loss == LOSS_POISSON) hipLaunchKernelGGL(re_tron_csr_kernel<1>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  else hipLaunchKernelGGL(re_tron_csr_kernel<2>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  LAUNCH_CHECK();
  return 0;
}

// Lean streaming kernel (dmax <= 1024): LDS (1 + RE_NW) x dmax doubles; ``gsc`` scratch of one double per
// coefficient (packed like W); W is updated in place.
size_t pml_re_tron_lean_smem(int dmax) { return ((size_t)(1 + LEAN_NW) * dmax + 2 * LEAN_NW * 8) * sizeof(double); }

int pml_re_tron_lean(const int* order, int n_launch, const long long* row_ptr, const long long* col_ptr,
                     const long long* nip, const uint16_t* lcol, const double* val, const double* y,
                     const double* off, const double* wt, double* scr, long long n_rows, double* W, double* f,
                     int* iters, int* reason, double* zout, int* npass, int loss, double l2, double tol,
                     int max_iter, int max_fail, int max_cg, int dmax, double* gsc, int quad, const double* xf2,
                     hipStream_t st) {
  if (n_launch <= 0) return 0;
  if (dmax <= 0 || dmax > 1024 || loss < 0 || loss > 2 || gsc == nullptr) return -22;
  const size_t smem = pml_re_tron_lean_smem(dmax);
  ReTronArgs a{order, n_launch, row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr, n_rows, W, f, iters, reason,
               zout, npass, loss, l2, tol, max_iter, max_fail, max_cg, dmax, gsc, xf2};
  // quad: every row padded to a multiple of 4 entries (row_pass_q), else the strided row_pass
  if (quad) {
    if (loss == LOSS_LOGISTIC) lean_launch<0, true>(a, n_launch, smem, st);
    else if (loss == LOSS_POISSON) lean_launch<1, true>(a, n_launch, smem, st);
    else lean_launch<2, true>(a, n_launch, smem, st);
  } else {
    if (loss == LOSS_LOGISTIC) lean_launch<0, false>(a, n_launch, smem, st);
    else if (loss == LOSS_POISSON) lean_launch<1, false>(a, n_launch, smem, st);
    else lean_launch<2, false>(a, n_launch, smem, st);
  }
  LAUNCH_CHECK();
  return 0;
}

// Tall-narrow entities (d_e <= 64): one wave (= one workgroup) per entity; LDS per workgroup.
size_t pml_re_tron_hess_smem(int dp) {
  switch (dp / 16) {
    case 1: return (size_t)TallCfg<1>::WORDS * sizeof(double);
    case 2: return (size_t)TallCfg<2>::WORDS * sizeof(double);
    case 3: return (size_t)TallCfg<3>::WORDS * sizeof(double);
    default: return (size_t)TallCfg<4>::WORDS * sizeof(double);
  }
}

int pml_re_tron_hess(const int* order, int n_launch, const long long* row_ptr, const long long* col_ptr,
                     const long long* nip, const uint16_t* lcol, const double* val, const double* y,
                     const double* off, const double* wt, double* scr, long long n_rows, double* W, double* f,
                     int* iters, int* reason, double* zout, int* npass, int loss, double l2, double tol,
                     int max_iter, int max_fail, int max_cg, int dp, hipStream_t st) {
  if (n_launch <= 0) return 0;
  if (dp < 16 || dp > 64 || dp % 16 || loss < 0 || loss > 2) return -22;
  const size_t smem = pml_re_tron_hess_smem(dp);
  ReTronArgs a{order, n_launch, row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr, n_rows, W, f, iters, reason,
               zout, npass, loss, l2, tol, max_iter, max_fail, max_cg, dp};
#define RT_LAUNCH_L(T, L)                                                                                  \
  hipLaunchKernelGGL((re_tron_tall_kernel<T, L>), dim3(n_launch), dim3(64), smem, st, a)
#define RT_LAUNCH(T)                                  \
  do {                                                \
    if (loss == LOSS_LOGISTIC) RT_LAUNCH_L(T, 0);     \
    else if (loss == LOSS_POISSON) RT_LAUNCH_L(T, 1); \
    else RT_LAUNCH_L(T, 2);                           \
  } while (0)
  switch (dp / 16) {
    case 1: RT_LAUNCH(1); break;
    case 2: RT_LAUNCH(2); break;
    case 3: RT_LAUNCH(3); break;
    default: RT_LAUNCH(4); break;
  }
#undef RT_LAUNCH
#undef RT_LAUNCH_L
  LAUNCH_CHECK();
  return 0;
}


// Register-resident kernel: LDS per workgroup, rows per workgroup.
static size_t res_smem(int S) {
  const size_t cap = (size_t)RS_NW * 4 * S;
  return ((size_t)(6 + RS_NW) * (RS_DMAX + 8) + 7 * cap + 2 * RS_NW * 8 + 16) * sizeof(double);
}
int pml_re_res_cap() { return RS_NW * 4 * RES_S; }
int pml_re_res_dmax() { return RS_DMAX; }
size_t pml_re_res_ws_doubles(int n_tickets) { return (size_t)n_tickets * 2 * (RS_DMAX + 8); }

// Persistent launch over ``n_tasks`` tasks (task_ent / task_t0 as in ResTasks); ``ticket`` (1 int), ``bar``
// (n_tasks unsigned) and ``err`` (1 int) are zeroed here on the stream; ``ws``: pml_re_res_ws_doubles(n_tickets).
int pml_re_tron_res(const int* task_ent, const int* task_t0, int n_tasks, int* ticket, unsigned* bar, double* ws,
                    int* err, int grid, const long long* row_ptr, const long long* col_ptr, const long long* nip,
                    const uint16_t* lcol, const double* val, const double* y, const double* off, const double* wt,
                    double* W, double* f, int* iters, int* reason, double* zout, int* npass, int loss, double l2,
                    double tol, int max_iter, int max_fail, int max_cg, hipStream_t st) {
  if (n_tasks <= 0) return 0;
  if (loss < 0 || loss > 2 || grid <= 0) return -22;
  const size_t smem = res_smem(RES_S);
  if (smem > 160 * 1024) return -22;
  if (hipMemsetAsync(ticket, 0, sizeof(int), st) != hipSuccess) return -5;
  if (hipMemsetAsync(bar, 0, sizeof(unsigned) * n_tasks, st) != hipSuccess) return -5;
  if (hipMemsetAsync(err, 0, sizeof(int), st) != hipSuccess) return -5;
  ReTronArgs a{nullptr, 0, row_ptr, col_ptr, nip, lcol, val, y, off, wt, nullptr, 0, W, f, iters, reason,
               zout, npass, loss, l2, tol, max_iter, max_fail, max_cg, RS_DMAX};
  ResTasks tk{ticket, task_ent, task_t0, n_tasks, bar, ws, err};
  if (loss == LOSS_LOGISTIC)
    hipLaunchKernelGGL((re_tron_res_kernel<RES_S, 0>), dim3(grid), dim3(RS_THREADS), smem, st, a, tk);
  else if (loss == LOSS_POISSON)
    hipLaunchKernelGGL((re_tron_res_kernel<RES_S, 1>), dim3(grid), dim3(RS_THREADS), smem, st, a, tk);
  else
    hipLaunchKernelGGL((re_tron_res_kernel<RES_S, 2>), dim3(grid), dim3(RS_THREADS), smem, st, a, tk);
  LAUNCH_CHECK();
  return 0;
}

// Workgroups of the resident kernel that fit on the device at once (occupancy API x CUs; 0 on error).
int pml_re_res_grid() {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)re_tron_res_kernel<RES_S, 0>, RS_THREADS,
                                                   res_smem(RES_S)) != hipSuccess) return 0;
  return cus * per;
}


// Row-space TRON for 64 < n <= 192 (one wave per problem, packed L in LDS).
int pml_rs_tron_big(int B, int n, const double* L, const double* y, const double* off, const double* wt,
                    double* beta, double* f, int* iters, int* reason, double* zout, int loss, double l2, double tol,
                    int max_iter, int max_fail, int max_cg, hipStream_t st) {
  if (B <= 0) return 0;
  if (n < 1 || n > 192 || loss < 0 || loss > 2) return -22;
  const size_t smem = ((size_t)n * (n + 1) / 2 + n) * sizeof(double);
  if (smem > 160 * 1024) return -22;
#define RSB(E, LS) hipLaunchKernelGGL((rs_tron_big_kernel<E, LS>), dim3(B), dim3(64), smem, st, B, n, L, y, off, wt, \
                                      beta, f, iters, reason, zout, l2, tol, max_iter, max_fail, max_cg)
#define RSB_E(E) do { if (loss == 0) RSB(E, 0); else if (loss == 1) RSB(E, 1); else RSB(E, 2); } while (0)
  if (n <= 64) RSB_E(1);
  else if (n <= 128) RSB_E(2);
  else RSB_E(3);
#undef RSB_E
#undef RSB
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
