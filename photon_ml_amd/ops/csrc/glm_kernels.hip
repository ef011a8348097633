// photon_ml_amd — CDNA4 (gfx950 / MI355X) kernels for GLM aggregation.
//
// One data structure serves both sparse directions: a "segmented stream" = entries grouped in contiguous
// segments (CSR: segment = row; row-chunked CSC: segment = column of one row chunk). Work is split into
// pre-computed BLOCKS of <= NB entries (built once on the host, the sparsity pattern is static during
// training), in the spirit of AMD's CSR-adaptive SpMV:
//   * normal block  : several whole segments; entries streamed with 16-B vector loads (8 entries / lane /
//                     round), products staged in LDS, then a segmented reduction with a group size chosen from the
//                     segment count (1..64 lanes per segment, shuffles inside one wave64) and a fused epilogue.
//   * piece block   : one NB-entry piece of a segment longer than NB; writes one fp64 partial. A combine
//                     kernel sums the pieces IN ORDER (no atomics -> bitwise deterministic) and runs the epilogue.
// Epilogues:
//   forward (CSR)   : margin z = x.w_eff + shift (+offset) -> pointwise loss (logistic/poisson/squared/hinge) ->
//                     per-row coefficient wt*l' (fed to the transpose pass), optional cached wt*l'' (TRON Hv),
//                     block partial sums of (wt*l, wt*l') in fp64.
//   transpose (CSC) : G[col] += sum(val * coef[row])  (or val^2 * coef for the Hessian diagonal); rows of one
//                     chunk are a 1M-row window, so the coef gathers stay resident in the XCD L2 / Infinity Cache.
// Reference semantics: photon-lib/.../function/glm/{ValueAndGradient,HessianVector,HessianDiagonal}Aggregator.scala.
//
// Built with: hipcc --offload-arch=gfx950 -O3 -shared -fPIC (see photon_ml_amd/ops/build.py). C ABI, loaded
// with ctypes after torch (one HIP runtime per process; torch tensors provide the memory, the caller the stream).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define NB 4096          // max entries per block
#define NTHREADS 256     // 4 wave64 per block
#define VEC 8            // entries per lane per load round
#define MAXSEG 2048      // max segments per normal block

enum LossId { LOSS_LOGISTIC = 0, LOSS_POISSON = 1, LOSS_SQUARED = 2, LOSS_HINGE = 3 };
enum FwdMode { FWD_MARGIN = 0, FWD_VALUE_GRAD = 1, FWD_HV = 2, FWD_DZZ = 3 };

// ------------------------------------------------------------------------------------------------------------
// value loads: 8 consecutive entries -> AT[8]
struct bf16x8 { uint4 u; };

template <typename VT, typename AT> struct Loader;
template <> struct Loader<uint16_t, float> {
  static __device__ __forceinline__ void load8(const uint16_t* __restrict__ p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(w[k] << 16);
      v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
};
template <> struct Loader<float, float> {
  static __device__ __forceinline__ void load8(const float* __restrict__ p, float* v) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};
template <> struct Loader<double, double> {
  static __device__ __forceinline__ void load8(const double* __restrict__ p, double* v) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double2 a = *reinterpret_cast<const double2*>(p + 2 * k);
      v[2 * k] = a.x; v[2 * k + 1] = a.y;
    }
  }
};

// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ double log1p_exp(double x) {
  return x > 0.0 ? x + log1p(exp(-x)) : log1p(exp(x));
}

// returns l, dl, d2l
__device__ __forceinline__ void pointwise_loss(int loss, double z, double y, double& l, double& dl, double& d2) {
  if (loss == LOSS_LOGISTIC) {
    double s = 1.0 / (1.0 + exp(-z));
    if (y > 0.5) { l = log1p_exp(-z); dl = s - 1.0; }
    else { l = log1p_exp(z); dl = s; }
    d2 = s * (1.0 - s);
  } else if (loss == LOSS_POISSON) {
    double e = exp(z);
    l = e - y * z; dl = e - y; d2 = e;
  } else if (loss == LOSS_SQUARED) {
    double d = z - y;
    l = 0.5 * d * d; dl = d; d2 = 1.0;
  } else {  // smoothed hinge
    double yy = y < 0.5 ? -1.0 : 1.0;
    double t = yy * z;
    l = t <= 0.0 ? 0.5 - t : (t < 1.0 ? 0.5 * (1.0 - t) * (1.0 - t) : 0.0);
    double d = t < 0.0 ? -1.0 : (t < 1.0 ? t - 1.0 : 0.0);
    dl = d * yy; d2 = 0.0;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of two doubles; result valid in thread 0
__device__ __forceinline__ void block_sum2(double& a, double& b, double* sh /*[2*NTHREADS/64]*/) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) { sh[2 * w] = a; sh[2 * w + 1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0; b = 0.0;
    for (int i = 0; i < NTHREADS / 64; ++i) { a += sh[2 * i]; b += sh[2 * i + 1]; }
  }
}

// Block descriptor: {seg_lo, seg_hi, nz_lo, nz_hi, part}; part >= 0 marks a piece of a long segment.
struct BlockDesc { int seg_lo, seg_hi, nz_lo, nz_hi, part; };

__device__ __forceinline__ BlockDesc load_desc(const int* __restrict__ blk, int b) {
  const int* p = blk + 5 * b;
  BlockDesc d; d.seg_lo = p[0]; d.seg_hi = p[1]; d.nz_lo = p[2]; d.nz_hi = p[3]; d.part = p[4];
  return d;
}

// Stream [lo8, hi8) (8-aligned window around [nz_lo, nz_hi)), computing products val*x[idx] (SQ: val^2*x[idx]).
// Normal blocks stage products into LDS; piece blocks return the thread's partial sum.
template <typename VT, typename XT, typename AT, bool SQ>
__device__ __forceinline__ double stream_products(const BlockDesc& d, const int* __restrict__ idx,
                                                  const VT* __restrict__ val, const XT* __restrict__ x,
                                                  AT* prod, bool to_lds) {
  const int lo = d.nz_lo & ~(VEC - 1);
  const int hi = (d.nz_hi + VEC - 1) & ~(VEC - 1);
  double acc = 0.0;
  for (int e = lo + threadIdx.x * VEC; e < hi; e += NTHREADS * VEC) {
    int4 i0 = *reinterpret_cast<const int4*>(idx + e);
    int4 i1 = *reinterpret_cast<const int4*>(idx + e + 4);
    int ii[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
    AT v[8];
    Loader<VT, AT>::load8(val + e, v);
    AT p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool in = (e + k >= d.nz_lo) && (e + k < d.nz_hi);
      const int j = in ? ii[k] : 0;
      AT xv = static_cast<AT>(x[j]);
      AT vv = SQ ? v[k] * v[k] : v[k];
      p[k] = in ? vv * xv : AT(0);
    }
    if (to_lds) {
#pragma unroll
      for (int k = 0; k < 8; ++k) prod[e - lo + k] = p[k];
    } else {
      float s4 = 0.f;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += static_cast<double>(p[k]);
      (void)s4;
      acc += s;
    }
  }
  return acc;
}

// Group size (lanes per segment) for the segmented reduction.
__device__ __forceinline__ int group_size(int nseg) {
  if (nseg <= 4) return 64;
  int g = NTHREADS / nseg;
  if (g >= 64) return 64;
  if (g >= 32) return 32;
  if (g >= 16) return 16;
  if (g >= 8) return 8;
  if (g >= 4) return 4;
  if (g >= 2) return 2;
  return 1;
}

template <typename AT>
__device__ __forceinline__ double group_reduce(double v, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------------------------------------
// Forward (CSR) epilogue arguments
template <typename XT, typename RT>
struct FwdArgs {
  int mode, loss;
  double shift;       // margin shift (-w_eff . s), or v_shift for HV
  const RT* y; const RT* off; const RT* wt;
  XT* coef;           // VALUE_GRAD: wt*l'; HV: e_i; DZZ: wt*l''
  XT* dzz;            // VALUE_GRAD with cache: wt*l''; HV: input D_i
  double* z_out;      // MARGIN: z (double)
  int with_offset;    // MARGIN: add offset
};

template <typename XT, typename RT>
__device__ __forceinline__ void fwd_epilogue(const FwdArgs<XT, RT>& a, int s, double sum, double& F, double& S) {
  if (a.mode == FWD_MARGIN) {
    double z = sum + a.shift;
    if (a.with_offset) z += static_cast<double>(a.off[s]);
    a.z_out[s] = z;
    return;
  }
  if (a.mode == FWD_HV) {
    double e = static_cast<double>(a.dzz[s]) * (sum - a.shift);
    a.coef[s] = static_cast<XT>(e);
    S += e;
    return;
  }
  const double z = sum + a.shift + static_cast<double>(a.off[s]);
  const double y = static_cast<double>(a.y[s]);
  const double w = static_cast<double>(a.wt[s]);
  double l, dl, d2;
  pointwise_loss(a.loss, z, y, l, dl, d2);
  if (a.mode == FWD_VALUE_GRAD) {
    a.coef[s] = static_cast<XT>(w * dl);
    if (a.dzz) a.dzz[s] = static_cast<XT>(w * d2);
    F += w * l;
    S += w * dl;
  } else {  // FWD_DZZ
    a.coef[s] = static_cast<XT>(w * d2);
  }
}

template <typename VT, typename XT, typename RT, typename AT>
__global__ __launch_bounds__(NTHREADS) void seg_fwd_kernel(
    const int* __restrict__ blk, const int* __restrict__ seg_ptr, const int* __restrict__ idx,
    const VT* __restrict__ val, const XT* __restrict__ x, FwdArgs<XT, RT> a, double* __restrict__ stats,
    double* __restrict__ parts) {
  __shared__ AT prod[NB + 2 * VEC];
  __shared__ double sh[2 * NTHREADS / 64];
  const BlockDesc d = load_desc(blk, blockIdx.x);
  if (d.part >= 0) {
    double acc = stream_products<VT, XT, AT, false>(d, idx, val, x, prod, false);
    double dummy = 0.0;
    block_sum2(acc, dummy, sh);
    if (threadIdx.x == 0) parts[d.part] = acc;
    if (threadIdx.x == 0 && stats) { stats[2 * blockIdx.x] = 0.0; stats[2 * blockIdx.x + 1] = 0.0; }
    return;
  }
  stream_products<VT, XT, AT, false>(d, idx, val, x, prod, true);
  __syncthreads();
  const int lo = d.nz_lo & ~(VEC - 1);
  const int nseg = d.seg_hi - d.seg_lo;
  const int G = group_size(nseg);
  const int gid = threadIdx.x / G, gl = threadIdx.x % G, ngroups = NTHREADS / G;
  double F = 0.0, S = 0.0;
  for (int base = 0; base < nseg; base += ngroups) {
    const int si = base + gid;
    double sum = 0.0;
    int s = -1;
    if (si < nseg) {
      s = d.seg_lo + si;
      const int b0 = seg_ptr[s] - lo, b1 = seg_ptr[s + 1] - lo;
      for (int j = b0 + gl; j < b1; j += G) sum += static_cast<double>(prod[j]);
    }
    sum = group_reduce<AT>(sum, G);
    if (si < nseg && gl == 0) fwd_epilogue(a, s, sum, F, S);
  }
  if (stats) {
    block_sum2(F, S, sh);
    if (threadIdx.x == 0) { stats[2 * blockIdx.x] = F; stats[2 * blockIdx.x + 1] = S; }
  }
}

// combine pieces of long forward segments: one wave per long segment, pieces summed lane-strided then tree
template <typename XT, typename RT>
__global__ __launch_bounds__(64) void seg_fwd_long_kernel(const int* __restrict__ long_seg,
                                                          const int* __restrict__ long_ptr,
                                                          const double* __restrict__ parts, FwdArgs<XT, RT> a,
                                                          double* __restrict__ long_stats) {
  const int L = blockIdx.x;
  const int p0 = long_ptr[L], p1 = long_ptr[L + 1];
  double sum = 0.0;
  for (int p = p0 + threadIdx.x; p < p1; p += 64) sum += parts[p];
  sum = wave_sum(sum);
  if (threadIdx.x == 0) {
    double F = 0.0, S = 0.0;
    fwd_epilogue(a, long_seg[L], sum, F, S);
    if (long_stats) { long_stats[2 * L] = F; long_stats[2 * L + 1] = S; }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Transpose (row-chunked CSC): G[col] += sum_i val * x[row]   (SQ: val^2)
template <typename VT, typename XT, typename AT, bool SQ>
__global__ __launch_bounds__(NTHREADS) void seg_t_kernel(const int* __restrict__ blk,
                                                         const int* __restrict__ seg_ptr,
                                                         const int* __restrict__ idx, const VT* __restrict__ val,
                                                         const XT* __restrict__ x, double* __restrict__ G,
                                                         double* __restrict__ parts) {
  __shared__ AT prod[NB + 2 * VEC];
  __shared__ double sh[2 * NTHREADS / 64];
  const BlockDesc d = load_desc(blk, blockIdx.x);
  if (d.part >= 0) {
    double acc = stream_products<VT, XT, AT, SQ>(d, idx, val, x, prod, false);
    double dummy = 0.0;
    block_sum2(acc, dummy, sh);
    if (threadIdx.x == 0) parts[d.part] = acc;
    return;
  }
  stream_products<VT, XT, AT, SQ>(d, idx, val, x, prod, true);
  __syncthreads();
  const int lo = d.nz_lo & ~(VEC - 1);
  const int nseg = d.seg_hi - d.seg_lo;
  const int G_ = group_size(nseg);
  const int gid = threadIdx.x / G_, gl = threadIdx.x % G_, ngroups = NTHREADS / G_;
  for (int base = 0; base < nseg; base += ngroups) {
    const int si = base + gid;
    double sum = 0.0;
    int s = -1, b0 = 0, b1 = 0;
    if (si < nseg) {
      s = d.seg_lo + si;
      b0 = seg_ptr[s] - lo; b1 = seg_ptr[s + 1] - lo;
      for (int j = b0 + gl; j < b1; j += G_) sum += static_cast<double>(prod[j]);
    }
    sum = group_reduce<AT>(sum, G_);
    if (si < nseg && gl == 0 && b1 > b0) G[s] += sum;
  }
}

__global__ __launch_bounds__(64) void seg_t_long_kernel(const int* __restrict__ long_seg,
                                                        const int* __restrict__ long_ptr,
                                                        const double* __restrict__ parts, double* __restrict__ G) {
  const int L = blockIdx.x;
  const int p0 = long_ptr[L], p1 = long_ptr[L + 1];
  double sum = 0.0;
  for (int p = p0 + threadIdx.x; p < p1; p += 64) sum += parts[p];
  sum = wave_sum(sum);
  if (threadIdx.x == 0) G[long_seg[L]] += sum;
}

// ------------------------------------------------------------------------------------------------------------
// Deterministic reduction of per-block (F, S) stats: out[0..1] (+)= sum. One workgroup.
__global__ __launch_bounds__(NTHREADS) void reduce_stats_kernel(const double* __restrict__ stats, int n,
                                                                 double* __restrict__ out, int accumulate) {
  __shared__ double sh[2 * NTHREADS / 64];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < n; i += NTHREADS) { a += stats[2 * i]; b += stats[2 * i + 1]; }
  block_sum2(a, b, sh);
  if (threadIdx.x == 0) {
    if (accumulate) { out[0] += a; out[1] += b; }
    else { out[0] = a; out[1] = b; }
  }
}

// Two-level deterministic reduction for large block counts: level 1 (grid of up to 256 WGs) -> partial pairs.
__global__ __launch_bounds__(NTHREADS) void reduce_stats_l1_kernel(const double* __restrict__ stats, int n,
                                                                    int per_wg, double* __restrict__ partial) {
  __shared__ double sh[2 * NTHREADS / 64];
  const int b0 = blockIdx.x * per_wg, b1 = min(n, b0 + per_wg);
  double a = 0.0, b = 0.0;
  for (int i = b0 + threadIdx.x; i < b1; i += NTHREADS) { a += stats[2 * i]; b += stats[2 * i + 1]; }
  block_sum2(a, b, sh);
  if (threadIdx.x == 0) { partial[2 * blockIdx.x] = a; partial[2 * blockIdx.x + 1] = b; }
}

// ============================================================================================================
// C ABI
// ============================================================================================================
// precision codes: 0 = bf16 values / f32 vectors / f32 row data; 1 = f32/f32/f32; 2 = f64/f64/f64
struct SegChunkDesc {
  const int* blk; int nblk;
  const int* seg_ptr; int nseg;
  const int* idx; const void* val;
  const int* long_seg; const int* long_ptr; int nlong; int npart;
};

#define LAUNCH_CHECK()                                         \
  do {                                                         \
    hipError_t e_ = hipGetLastError();                         \
    if (e_ != hipSuccess) return (int)e_;                      \
  } while (0)

template <typename VT, typename XT, typename RT, typename AT>
static int fwd_impl(const SegChunkDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats, double* long_stats,
                    double* parts, hipStream_t st) {
  if (c->nblk > 0) {
    hipLaunchKernelGGL((seg_fwd_kernel<VT, XT, RT, AT>), dim3(c->nblk), dim3(NTHREADS), 0, st, c->blk,
                       c->seg_ptr, c->idx, (const VT*)c->val, (const XT*)x, a, stats, parts);
    LAUNCH_CHECK();
  }
  if (c->nlong > 0) {
    hipLaunchKernelGGL((seg_fwd_long_kernel<XT, RT>), dim3(c->nlong), dim3(64), 0, st, c->long_seg, c->long_ptr,
                       parts, a, long_stats);
    LAUNCH_CHECK();
  }
  return 0;
}

template <typename VT, typename XT, typename AT, bool SQ>
static int t_impl(const SegChunkDesc* c, const void* x, double* G, double* parts, hipStream_t st) {
  if (c->nblk > 0) {
    hipLaunchKernelGGL((seg_t_kernel<VT, XT, AT, SQ>), dim3(c->nblk), dim3(NTHREADS), 0, st, c->blk, c->seg_ptr,
                       c->idx, (const VT*)c->val, (const XT*)x, G, parts);
    LAUNCH_CHECK();
  }
  if (c->nlong > 0) {
    hipLaunchKernelGGL(seg_t_long_kernel, dim3(c->nlong), dim3(64), 0, st, c->long_seg, c->long_ptr, parts, G);
    LAUNCH_CHECK();
  }
  return 0;
}

extern "C" {

int pml_version() { return 1; }
int pml_nb() { return NB; }
int pml_maxseg() { return MAXSEG; }

// ---- host-side block construction (greedy, sequential; the pattern is static so this runs once) ----------
// seg_ptr: int32[nseg+1] (host). Outputs sized by a first call with blk == NULL.
int pml_build_blocks(const int* seg_ptr, int nseg, int nb, int maxseg, int* blk, int* nblk_out,
                     int* long_seg, int* long_ptr, int* nlong_out, int* npart_out) {
  int nblk = 0, nlong = 0, npart = 0;
  int s = 0;
  if (long_ptr) long_ptr[0] = 0;
  while (s < nseg) {
    int len = seg_ptr[s + 1] - seg_ptr[s];
    if (len > nb) {
      // long segment -> pieces
      int np = (len + nb - 1) / nb;
      for (int p = 0; p < np; ++p) {
        if (blk) {
          int* q = blk + 5 * nblk;
          q[0] = s; q[1] = s + 1;
          q[2] = seg_ptr[s] + p * nb;
          q[3] = (p == np - 1) ? seg_ptr[s + 1] : seg_ptr[s] + (p + 1) * nb;
          q[4] = npart + p;
        }
        ++nblk;
      }
      if (long_seg) long_seg[nlong] = s;
      npart += np;
      ++nlong;
      if (long_ptr) long_ptr[nlong] = npart;
      ++s;
      continue;
    }
    // normal block: pack segments while entries (incl. alignment slack) fit NB
    int s0 = s;
    int base = seg_ptr[s0] & ~(VEC - 1);
    while (s < nseg && (s - s0) < maxseg) {
      int l = seg_ptr[s + 1] - seg_ptr[s];
      if (l > nb) break;
      int end_aligned = (seg_ptr[s + 1] + VEC - 1) & ~(VEC - 1);
      if (end_aligned - base > nb && s > s0) break;
      ++s;
    }
    if (blk) {
      int* q = blk + 5 * nblk;
      q[0] = s0; q[1] = s; q[2] = seg_ptr[s0]; q[3] = seg_ptr[s]; q[4] = -1;
    }
    ++nblk;
  }
  *nblk_out = nblk; *nlong_out = nlong; *npart_out = npart;
  return 0;
}

// Forward pass over one chunk. Row-data pointers (y/off/wt/coef/dzz/z_out) must already be offset to the
// chunk's first row. stats: double[2*nblk] (may be NULL for MARGIN/DZZ); long_stats: double[2*nlong];
// parts: double[npart] scratch.
int pml_seg_fwd(int prec, const SegChunkDesc* c, const void* x, int mode, int loss, double shift,
                const void* y, const void* off, const void* wt, void* coef, void* dzz, double* z_out,
                int with_offset, double* stats, double* long_stats, double* parts, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) {
    FwdArgs<double, double> a{mode, loss, shift, (const double*)y, (const double*)off, (const double*)wt,
                              (double*)coef, (double*)dzz, z_out, with_offset};
    return fwd_impl<double, double, double, double>(c, x, a, stats, long_stats, parts, st);
  }
  FwdArgs<float, float> a{mode, loss, shift, (const float*)y, (const float*)off, (const float*)wt,
                          (float*)coef, (float*)dzz, z_out, with_offset};
  if (prec == 1) return fwd_impl<float, float, float, float>(c, x, a, stats, long_stats, parts, st);
  return fwd_impl<uint16_t, float, float, float>(c, x, a, stats, long_stats, parts, st);
}


// Transpose pass over one CSC chunk: G[col] += sum val*x[row] (square=1: val^2). x is offset by caller so that
// local row r of this chunk reads x[r].
int pml_seg_t(int prec, const SegChunkDesc* c, const void* x, int square, double* G, double* parts, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) {
    return square ? t_impl<double, double, double, true>(c, x, G, parts, st)
                  : t_impl<double, double, double, false>(c, x, G, parts, st);
  }
  if (prec == 1) {
    return square ? t_impl<float, float, float, true>(c, x, G, parts, st)
                  : t_impl<float, float, float, false>(c, x, G, parts, st);
  }
  return square ? t_impl<uint16_t, float, float, true>(c, x, G, parts, st)
                : t_impl<uint16_t, float, float, false>(c, x, G, parts, st);
}

// out[0..1] (+)= sum of n (F,S) pairs. scratch: >= 2*256 doubles. Deterministic for fixed n.
int pml_reduce_stats(const double* stats, int n, double* out, int accumulate, double* scratch, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0) return 0;
  if (n <= 8192 || scratch == nullptr) {
    hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(NTHREADS), 0, st, stats, n, out, accumulate);
    LAUNCH_CHECK();
    return 0;
  }
  const int nwg = 256;
  const int per = (n + nwg - 1) / nwg;
  hipLaunchKernelGGL(reduce_stats_l1_kernel, dim3(nwg), dim3(NTHREADS), 0, st, stats, n, per, scratch);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(NTHREADS), 0, st, scratch, nwg, out, accumulate);
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
