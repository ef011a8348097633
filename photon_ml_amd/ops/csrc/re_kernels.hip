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

#define LAUNCH_CHECK()                                         \
  do {                                                         \
    hipError_t e_ = hipGetLastError();                         \
    if (e_ != hipSuccess) return (int)e_;                      \
  } while (0)

#define RE_NW 4                 // waves per workgroup (one entity)
#define RE_THREADS (RE_NW * 64)
#define RE_R 4                  // rows in flight per wave

enum { LOSS_LOGISTIC = 0, LOSS_POISSON = 1, LOSS_SQUARED = 2 };

__device__ __forceinline__ double log1p_exp(double x) { return x > 0.0 ? x + log1p(exp(-x)) : log1p(exp(x)); }

__device__ __forceinline__ void pointwise_loss(int loss, double z, double y, double& l, double& dl, double& d2) {
  if (loss == LOSS_LOGISTIC) {
    const double s = 1.0 / (1.0 + exp(-z));
    if (y > 0.5) { l = log1p_exp(-z); dl = s - 1.0; }
    else { l = log1p_exp(z); dl = s; }
    d2 = s * (1.0 - s);
  } else if (loss == LOSS_POISSON) {
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

// Workgroup sums of K values (K <= 8), in every thread. ``red`` holds two [RE_NW][8] slots used alternately,
// so one barrier per call suffices: a slot is rewritten only two calls later, after every thread has passed
// the barrier of the call in between (all threads run the same, workgroup-uniform control flow).
template <int K>
__device__ __forceinline__ void block_sums(double (&v)[K], double* __restrict__ red, int& parity) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_total(v[k]);
  double* slot = red + parity * (RE_NW * 8);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) slot[w * 8 + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < RE_NW; ++q) s += slot[q * 8 + k];
    v[k] = s;
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
};

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
#define RE_U 3                       // instruction groups in flight per wave batch
#define RE_BATCH (RE_RPI * RE_U)     // rows per wave batch
#define RE_K 4                       // entries per lane kept in registers (rows of <= 64 entries in one go)

// One pass over the entity's rows [r0, r1): a wave takes RE_BATCH consecutive rows at a time, RE_G lanes per
// row (lane k of the row: entries k, k + 16, ...). The next batch's row pointers are fetched while the current
// batch computes, and all RE_BATCH rows' entries are loaded before the first gather, so a batch costs about one
// dependent global-memory latency.
// MODE 0: Hessian-vector data term: acc_w += X^T (Dc * (X vec)).
// MODE 1: value + gradient at vec: acc_w += X^T (wt * l'), fpart += wt * l, Dn = wt * l'', Zn = x.vec.
// MODE 2: value + gradient at zero (no gathers, no scratch writes).
template <int MODE>
__device__ __forceinline__ void row_pass(const ReTronArgs& a, long long r0, long long r1,
                                         const double* __restrict__ vec, double* __restrict__ acc,
                                         const double* __restrict__ Dc, double* __restrict__ Dn,
                                         double* __restrict__ Zn, double& fpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / RE_G, gl = lane % RE_G;
  const long long step = (long long)RE_NW * RE_BATCH;
  long long base = r0 + (long long)w * RE_BATCH;
  // row pointers of a batch: lane j <= RE_BATCH holds nip[base + j] (clamped to the entity's last row)
  auto fetch_ptr = [&](long long b) -> long long {
    const long long i = b + (lane <= RE_BATCH ? lane : RE_BATCH);
    return b < r1 ? a.nip[i < r1 ? i : r1] : 0;
  };
  long long np = fetch_ptr(base);
  for (; base < r1; base += step) {
    const long long np_next = fetch_ptr(base + step);
    long long lo[RE_U], hi[RE_U];
    int c[RE_U][RE_K];
    double v[RE_U][RE_K], dot[RE_U], rs[RE_U][3];
#pragma unroll
    for (int u = 0; u < RE_U; ++u) {
      const int q = u * RE_RPI + grp;
      lo[u] = __shfl(np, q, 64);
      hi[u] = __shfl(np, q + 1, 64);
      const long long i = base + q;
      const bool valid = i < r1;
      if (MODE == 0) {
        rs[u][0] = valid ? Dc[i] : 0.0;
      } else {
        rs[u][0] = valid ? a.wt[i] : 0.0;
        rs[u][1] = valid ? a.off[i] : 0.0;
        rs[u][2] = valid ? a.y[i] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < RE_U; ++u) {
#pragma unroll
      for (int k = 0; k < RE_K; ++k) {
        const long long p = lo[u] + gl + RE_G * k;
        const bool in = p < hi[u];
        c[u][k] = in ? (int)a.lcol[p] : 0;
        v[u][k] = in ? a.val[p] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < RE_U; ++u) {
      double s = 0.0;
      if (MODE != 2) {
#pragma unroll
        for (int k = 0; k < RE_K; ++k) s = fma(v[u][k], vec[c[u][k]], s);
        for (long long p = lo[u] + gl + RE_G * RE_K; p < hi[u]; p += RE_G) s = fma(a.val[p], vec[a.lcol[p]], s);
      }
      dot[u] = s;
    }
#pragma unroll
    for (int u = 0; u < RE_U; ++u) {
      if (MODE != 2) dot[u] = row16_total(dot[u]);
      const long long i = base + u * RE_RPI + grp;
      const bool valid = i < r1;
      double t;
      if (MODE == 0) {
        t = rs[u][0] * dot[u];
      } else {
        double l = 0.0, dl = 0.0, d2 = 0.0;
        if (valid) {
          pointwise_loss(a.loss, dot[u] + rs[u][1], rs[u][2], l, dl, d2);
          if (gl == 0) {
            fpart += rs[u][0] * l;
            if (MODE == 1) { Dn[i] = rs[u][0] * d2; Zn[i] = dot[u]; }
          }
        }
        t = rs[u][0] * dl;
      }
#pragma unroll
      for (int k = 0; k < RE_K; ++k)
        if (lo[u] + gl + RE_G * k < hi[u]) atomicAdd(&acc[c[u][k]], t * v[u][k]);
      for (long long p = lo[u] + gl + RE_G * RE_K; p < hi[u]; p += RE_G) atomicAdd(&acc[a.lcol[p]], t * a.val[p]);
    }
    np = np_next;
  }
}

// Variant 3: the batch loop software-pipelined — while batch b computes (LDS gathers, DPP sums, loss, LDS
// scatters) the entries of batch b + 1 are already in flight, so a wave keeps memory requests outstanding through
// its arithmetic instead of alternating load / compute. Two register slots of RE_U3 row groups each.
#define RE_U3 2
#define RE_BATCH3 (RE_RPI * RE_U3)
template <int MODE>
__device__ __forceinline__ void row_pass_pipe(const ReTronArgs& a, long long r0, long long r1,
                                              const double* __restrict__ vec, double* __restrict__ acc,
                                              const double* __restrict__ Dc, double* __restrict__ Dn,
                                              double* __restrict__ Zn, double& fpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = lane / RE_G, gl = lane % RE_G;
  const long long step = (long long)RE_NW * RE_BATCH3;
  struct Slot {
    long long base, lo[RE_U3], hi[RE_U3];
    int c[RE_U3][RE_K];
    double v[RE_U3][RE_K], rs[RE_U3][3];
  };
  auto fetch_ptr = [&](long long b) -> long long {
    const long long i = b + (lane <= RE_BATCH3 ? lane : RE_BATCH3);
    return b < r1 ? a.nip[i < r1 ? i : r1] : 0;
  };
  auto load = [&](Slot& sl, long long b, long long np) {
    sl.base = b;
#pragma unroll
    for (int u = 0; u < RE_U3; ++u) {
      const int q = u * RE_RPI + grp;
      sl.lo[u] = __shfl(np, q, 64);
      sl.hi[u] = __shfl(np, q + 1, 64);
      const long long i = b + q;
      const bool valid = i < r1;
      if (MODE == 0) {
        sl.rs[u][0] = valid ? Dc[i] : 0.0;
      } else {
        sl.rs[u][0] = valid ? a.wt[i] : 0.0;
        sl.rs[u][1] = valid ? a.off[i] : 0.0;
        sl.rs[u][2] = valid ? a.y[i] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < RE_K; ++k) {
        const long long p = sl.lo[u] + gl + RE_G * k;
        const bool in = p < sl.hi[u];
        sl.c[u][k] = in ? (int)a.lcol[p] : 0;
        sl.v[u][k] = in ? a.val[p] : 0.0;
      }
    }
  };
  auto process = [&](const Slot& sl) {
#pragma unroll
    for (int u = 0; u < RE_U3; ++u) {
      double dot = 0.0;
      if (MODE != 2) {
#pragma unroll
        for (int k = 0; k < RE_K; ++k) dot = fma(sl.v[u][k], vec[sl.c[u][k]], dot);
        for (long long p = sl.lo[u] + gl + RE_G * RE_K; p < sl.hi[u]; p += RE_G) dot = fma(a.val[p], vec[a.lcol[p]], dot);
        dot = row16_total(dot);
      }
      const long long i = sl.base + u * RE_RPI + grp;
      const bool valid = i < r1;
      double t;
      if (MODE == 0) {
        t = sl.rs[u][0] * dot;
      } else {
        double l = 0.0, dl = 0.0, d2 = 0.0;
        if (valid) {
          pointwise_loss(a.loss, dot + sl.rs[u][1], sl.rs[u][2], l, dl, d2);
          if (gl == 0) {
            fpart += sl.rs[u][0] * l;
            if (MODE == 1) { Dn[i] = sl.rs[u][0] * d2; Zn[i] = dot; }
          }
        }
        t = sl.rs[u][0] * dl;
      }
#pragma unroll
      for (int k = 0; k < RE_K; ++k)
        if (sl.lo[u] + gl + RE_G * k < sl.hi[u]) atomicAdd(&acc[sl.c[u][k]], t * sl.v[u][k]);
      for (long long p = sl.lo[u] + gl + RE_G * RE_K; p < sl.hi[u]; p += RE_G)
        atomicAdd(&acc[a.lcol[p]], t * a.val[p]);
    }
  };
  long long base = r0 + (long long)w * RE_BATCH3;
  if (base >= r1) return;
  Slot A, B;
  long long np = fetch_ptr(base);
  load(A, base, np);
  np = fetch_ptr(base + step);
  for (;; base += 2 * step) {
    // A holds batch `base`; B gets batch base + step while A computes
    const bool hasB = base + step < r1;
    if (hasB) load(B, base + step, np);
    np = fetch_ptr(base + 2 * step);
    process(A);
    if (!hasB) break;
    const bool hasA = base + 2 * step < r1;
    if (hasA) load(A, base + 2 * step, np);
    np = fetch_ptr(base + 3 * step);
    process(B);
    if (!hasA) break;
  }
}

// Previous row pass (wave per row, lane = entry; one row's entries per instruction) — kept for A/B
// (PML_RE_ROWPASS=1).
template <int MODE>
__device__ __forceinline__ void row_pass_v1(const ReTronArgs& a, long long r0, long long r1,
                                            const double* __restrict__ vec, double* __restrict__ acc,
                                            const double* __restrict__ Dc, double* __restrict__ Dn,
                                            double* __restrict__ Zn, double& fpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (long long base = r0 + (long long)w * RE_R; base < r1; base += (long long)RE_NW * RE_R) {
    long long lo[RE_R], hi[RE_R];
    int c[RE_R];
    double v[RE_R], dot[RE_R], t[RE_R];
#pragma unroll
    for (int q = 0; q < RE_R; ++q) {
      const long long i = base + q;
      lo[q] = i < r1 ? a.nip[i] : 0;
      hi[q] = i < r1 ? a.nip[i + 1] : 0;
    }
#pragma unroll
    for (int q = 0; q < RE_R; ++q) {
      const long long p = lo[q] + lane;
      const bool in = p < hi[q];
      c[q] = in ? (int)a.lcol[p] : 0;
      v[q] = in ? a.val[p] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < RE_R; ++q) {
      dot[q] = MODE == 2 ? 0.0 : v[q] * vec[c[q]];
      if (MODE != 2) {
        for (long long p = lo[q] + 64 + lane; p < hi[q]; p += 64) dot[q] = fma(a.val[p], vec[a.lcol[p]], dot[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < RE_R; ++q) {
      if (MODE != 2) dot[q] = wave_total(dot[q]);
      const long long i = base + q;
      const bool valid = i < r1;
      if (MODE == 0) {
        t[q] = valid ? Dc[i] * dot[q] : 0.0;
      } else {
        double l = 0.0, dl = 0.0, d2 = 0.0, wi = 0.0;
        if (valid) {
          wi = a.wt[i];
          pointwise_loss(a.loss, dot[q] + a.off[i], a.y[i], l, dl, d2);
          if (lane == 0) {
            fpart += wi * l;
            if (MODE == 1) { Dn[i] = wi * d2; Zn[i] = dot[q]; }
          }
        }
        t[q] = wi * dl;
      }
    }
#pragma unroll
    for (int q = 0; q < RE_R; ++q) {
      if (lo[q] + lane < hi[q]) atomicAdd(&acc[c[q]], t[q] * v[q]);
      for (long long p = lo[q] + 64 + lane; p < hi[q]; p += 64) atomicAdd(&acc[a.lcol[p]], t[q] * a.val[p]);
    }
  }
}

template <int MODE, int V>
__device__ __forceinline__ void rows(const ReTronArgs& a, long long r0, long long r1, const double* vec, double* acc,
                                     const double* Dc, double* Dn, double* Zn, double& fpart) {
  if constexpr (V == 1) row_pass_v1<MODE>(a, r0, r1, vec, acc, Dc, Dn, Zn, fpart);
  else if constexpr (V == 3) row_pass_pipe<MODE>(a, r0, r1, vec, acc, Dc, Dn, Zn, fpart);
  else row_pass<MODE>(a, r0, r1, vec, acc, Dc, Dn, Zn, fpart);
}

template <int V>
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
    if (at_zero) rows<2, V>(a, r0, r1, vec, myacc, nullptr, nullptr, nullptr, fp);
    else rows<1, V>(a, r0, r1, vec, myacc, nullptr, D[nb], Z[nb], fp);
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
      rows<0, V>(a, r0, r1, sD, myacc, D[cur], nullptr, nullptr, fp);
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

// ============================================================================================================
// Tall-narrow entities (more rows than coefficients, d_e <= 64): TRON with the EXACT per-entity Hessian
// H_e = X_e^T D X_e + l2 I formed once per outer iteration on the fp64 MATRIX CORES and kept in LDS; every
// truncated-CG step is then a d_e x d_e LDS mat-vec instead of a pass over the entity's rows (per outer iteration:
// one Hessian pass + one function evaluation, against 1 + #CG passes for re_tron_csr_kernel).
// Hessian pass: rows are staged 64 at a time as a dense [64 x DP] LDS block (DP = d_e padded to 16) with their
// weights D_i; the upper-triangle 16 x 16 tiles of H are spread over the 4 waves, and per group of 4 staged rows
// every tile takes one v_mfma_f64_16x16x4f64: A[r][k] = X[k][16 ti + r], B[k][c] = D_k X[k][16 tj + c]
// (lane l: r = c = l & 15, k = l >> 4; accumulator i of lane l holds C[(l >> 4) + 4 i][l & 15]). Fixed k order
// per tile, each tile owned by one wave: deterministic. Diagonal tiles are stored as computed (not mirrored:
// C[r][c] and C[c][r] round differently), off-diagonal tiles into both halves.
// ============================================================================================================
typedef double v4d __attribute__((ext_vector_type(4)));
#define RH_ROWS 64

template <int T>
__global__ __launch_bounds__(RE_THREADS) void re_tron_hess_kernel(ReTronArgs a) {
  constexpr int DP = 16 * T;
  constexpr int NT = T * (T + 1) / 2;                 // upper-triangle tiles
  constexpr int NTW = (NT + RE_NW - 1) / RE_NW;       // tiles per wave (at most)
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int e = a.order[blockIdx.x];
  const long long r0 = a.row_ptr[e], r1 = a.row_ptr[e + 1];
  const long long c0 = a.col_ptr[e];
  const int d = (int)(a.col_ptr[e + 1] - c0);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  double* H = smem;                       // [DP][DP]
  double* Xs = H + DP * DP;               // [RH_ROWS][DP] staged rows
  double* Ds = Xs + RH_ROWS * DP;         // [RH_ROWS] their Hessian weights
  double* sW = Ds + RH_ROWS;
  double* sG = sW + DP;
  double* sS = sG + DP;
  double* sR = sS + DP;
  double* sD = sR + DP;
  double* acc = sD + DP;                  // RE_NW accumulators of DP (function evaluations), acc[0..d) = result
  double* red = acc + RE_NW * DP;
  double* myacc = acc + w * DP;
  double* D[2] = {a.scr, a.scr + a.n_rows};
  double* Z[2] = {a.scr + 2 * a.n_rows, a.scr + 3 * a.n_rows};
  int cur = 0, parity = 0, npass = 0;
  double* Wg = a.W + c0;
  // this wave's tiles (ti, tj), tj >= ti, round-robin over the waves
  int tI[NTW], tJ[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    int t = w + RE_NW * q, ti = 0;
    tI[q] = -1; tJ[q] = -1;
    if (t < NT) {
      while (t >= T - ti) { t -= T - ti; ++ti; }
      tI[q] = ti; tJ[q] = ti + t;
    }
  }
  auto zero_own = [&]() {
    for (int j = lane; j < d; j += 64) myacc[j] = 0.0;
  };
  auto value_grad = [&](const double* vec, int nb, bool at_zero, double& gg) -> double {
    ++npass;
    __syncthreads();
    zero_own();
    double fp = 0.0;
    if (at_zero) rows<2, 2>(a, r0, r1, vec, myacc, nullptr, nullptr, nullptr, fp);
    else rows<1, 2>(a, r0, r1, vec, myacc, nullptr, D[nb], Z[nb], fp);
    __syncthreads();
    double s3[3] = {fp, 0.0, 0.0};
    for (int j = tid; j < d; j += RE_THREADS) {
      double g = acc[j];
#pragma unroll
      for (int q = 1; q < RE_NW; ++q) g += acc[q * DP + j];
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
  // H = X^T diag(D[cur]) X + l2 I on the matrix cores
  auto form_hessian = [&]() {
    ++npass;
    const double* Dc = D[cur];
    v4d cacc[NTW];
#pragma unroll
    for (int q = 0; q < NTW; ++q) cacc[q] = v4d{0.0, 0.0, 0.0, 0.0};
    for (long long base = r0; base < r1; base += RH_ROWS) {
      __syncthreads();
      for (int j = tid; j < RH_ROWS * DP; j += RE_THREADS) Xs[j] = 0.0;
      if (tid < RH_ROWS) Ds[tid] = base + tid < r1 ? Dc[base + tid] : 0.0;
      __syncthreads();
      for (int rr = w; rr < RH_ROWS; rr += RE_NW) {
        const long long i = base + rr;
        if (i >= r1) break;
        for (long long p = a.nip[i] + lane; p < a.nip[i + 1]; p += 64) Xs[rr * DP + (int)a.lcol[p]] = a.val[p];
      }
      __syncthreads();
      const int r = lane & 15;
#pragma unroll 4
      for (int kg = 0; kg < RH_ROWS / 4; ++kg) {
        const int k = kg * 4 + (lane >> 4);
        const double dk = Ds[k];
        const double* xk = Xs + k * DP;
#pragma unroll
        for (int q = 0; q < NTW; ++q) {
          if (tI[q] < 0) continue;
          const double av = xk[tI[q] * 16 + r];
          const double bv = dk * xk[tJ[q] * 16 + r];
          cacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, cacc[q], 0, 0, 0);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NTW; ++q) {
      if (tI[q] < 0) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = tI[q] * 16 + (lane >> 4) + 4 * i, col = tJ[q] * 16 + (lane & 15);
        H[row * DP + col] = cacc[q][i];
        if (tI[q] != tJ[q]) H[col * DP + row] = cacc[q][i];
      }
    }
    __syncthreads();
    if (tid < d) H[tid * DP + tid] += a.l2;
    __syncthreads();
  };

  for (int j = tid; j < DP; j += RE_THREADS) sW[j] = j < d ? Wg[j] : 0.0;
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
    for (int j = tid; j < DP; j += RE_THREADS) sS[j] = 0.0;
    double g0;
    f0z = value_grad(sS, 0, true, g0);
    g0n = sqrt(g0);
  }
  const double loss_tol = f0z * a.tol, grad_tol = g0n * a.tol;
  double delta = sqrt(gnorm2);
  int it = 0, fails = 0, reason = 0;
  bool active = true, need_h = true;
  if (delta == 0.0) { reason = 4; active = false; }
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, sg1 = 0.25, sg2 = 0.5, sg3 = 4.0;
  const int guard_max = a.max_iter * (a.max_fail + 1) + 5;
  for (int guard = 0; active && guard < guard_max; ++guard) {
    if (need_h) { form_hessian(); need_h = false; }
    for (int j = tid; j < DP; j += RE_THREADS) {
      sS[j] = 0.0;
      const double gj = j < d ? sG[j] : 0.0;
      sR[j] = -gj;
      sD[j] = -gj;
    }
    double rtr = gnorm2, sts = 0.0;
    const double cg_tol2 = 0.01 * gnorm2;
    for (int k = 0; k < a.max_cg; ++k) {
      if (!(rtr > cg_tol2)) break;
      __syncthreads();
      double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      for (int j = tid; j < d; j += RE_THREADS) {
        const double* hr = H + j * DP;
        double h0 = 0.0, h1 = 0.0;
        int c = 0;
        for (; c + 1 < d; c += 2) { h0 = fma(hr[c], sD[c], h0); h1 = fma(hr[c + 1], sD[c + 1], h1); }
        if (c < d) h0 = fma(hr[c], sD[c], h0);
        const double h = h0 + h1, dj = sD[j];
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
      __syncthreads();          // every row of H . d read sD before it changes
      for (int j = tid; j < d; j += RE_THREADS) {
        const double dj = sD[j];
        sS[j] += al * dj;
        const double rj = sR[j] - al * acc[j];
        sR[j] = rj;
        if (!hit) sD[j] = rj + beta * dj;
      }
      if (hit) break;
      rtr = rn;
      sts = tn;
    }
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
    const double fn = value_grad(sD, cur ^ 1, false, gn2);
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
      need_h = true;
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

static int g_re_variant = 2;   // row pass: 2 = 16 lanes per row, batched (default); 3 = the same, software-pipelined;
                               // 1 = one row per wave

extern "C" {

void pml_re_set_variant(int v) { g_re_variant = (v == 1 || v == 3) ? v : 2; }

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
  if (g_re_variant == 1) hipLaunchKernelGGL(re_tron_csr_kernel<1>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  else if (g_re_variant == 3) hipLaunchKernelGGL(re_tron_csr_kernel<3>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  else hipLaunchKernelGGL(re_tron_csr_kernel<2>, dim3(n_launch), dim3(RE_THREADS), smem, st, a);
  LAUNCH_CHECK();
  return 0;
}

// Tall-narrow entities (d_e <= 64): LDS = H + staged rows + their weights + 5 vectors + accumulators + sums.
size_t pml_re_tron_hess_smem(int dp) {
  return ((size_t)dp * dp + (size_t)RH_ROWS * dp + RH_ROWS + (5 + RE_NW) * (size_t)dp + 2 * RE_NW * 8) * sizeof(double);
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
  switch (dp / 16) {
    case 1: hipLaunchKernelGGL(re_tron_hess_kernel<1>, dim3(n_launch), dim3(RE_THREADS), smem, st, a); break;
    case 2: hipLaunchKernelGGL(re_tron_hess_kernel<2>, dim3(n_launch), dim3(RE_THREADS), smem, st, a); break;
    case 3: hipLaunchKernelGGL(re_tron_hess_kernel<3>, dim3(n_launch), dim3(RE_THREADS), smem, st, a); break;
    default: hipLaunchKernelGGL(re_tron_hess_kernel<4>, dim3(n_launch), dim3(RE_THREADS), smem, st, a); break;
  }
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
