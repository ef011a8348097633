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
#include <algorithm>

#define NB 4096          // max entries per block
#define NTHREADS 256     // 4 wave64 per block
#define VEC 8            // entries per lane per load round
#define MAXSEG 1024      // max segments per normal block

#define LAUNCH_CHECK()                                         \
  do {                                                         \
    hipError_t e_ = hipGetLastError();                         \
    if (e_ != hipSuccess) return (int)e_;                      \
  } while (0)

enum LossId { LOSS_LOGISTIC = 0, LOSS_POISSON = 1, LOSS_SQUARED = 2, LOSS_HINGE = 3 };
enum FwdMode { FWD_MARGIN = 0, FWD_VALUE_GRAD = 1, FWD_HV = 2, FWD_DZZ = 3, FWD_LS = 4 };

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
    // one exp, one log1p, one reciprocal: e = exp(-|z|) serves the sigmoid and both log(1 + exp(+-z))
    // (log1p_exp(x) = max(x, 0) + log1p(exp(-|x|)), bit-identical to log1p_exp)
    const double e = exp(-fabs(z));
    const double lp = log1p(e);
    const double r = 1.0 / (1.0 + e);
    const double s = z >= 0.0 ? r : e * r;
    if (y > 0.5) { l = (z < 0.0 ? -z : 0.0) + lp; dl = s - 1.0; }
    else { l = (z > 0.0 ? z : 0.0) + lp; dl = s; }
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

// weight x per-row term with an exact 0 for zero-weight rows whatever the term (down-sampled rows, row-sampled
// copies whose dropped rows carry partial margins: an overflowed exp must not turn 0 x inf into NaN)
__device__ __forceinline__ double wx(double w, double x) { return w != 0.0 ? w * x : 0.0; }

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

// ------------------------------------------------------------------------------------------------------------
// Streaming a block's window [lo8, hi8) (8-aligned around [nz_lo, nz_hi)) and forming products val * x[idx]
// (SQ: val^2 * x[idx]). Two lane layouts:
//   VECTOR  : lane owns 8 consecutive entries per round (16-B index/value loads).
//   STRIDED : entry = round*256 + lane, i.e. one wave-instruction touches 64 CONSECUTIVE entries. Index loads are
//             4 B/lane but still fully coalesced (256 B per wave-instruction); the gain is on the GATHERS: in a hot
//             CSC column consecutive entries are nearby rows, so one gather instruction hits a handful of cache
//             lines instead of 64 (the vector layout spreads an instruction's lanes over 512 entries).
// All of a block's stream loads are issued first (non-temporal: read once per pass, keep L1/L2 for the gathered
// vector), then all gathers, then the products. HOT: indices < hot_n are served from an LDS copy of the head of
// x (features relabelled by frequency, so the head is the hottest features).
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

// Streaming loads through an explicit GLOBAL address-space pointer. Stream pointers that are themselves loaded
// from memory (per-chunk pointer tables of the shard-wide kernels) would otherwise compile to FLAT loads, which
// count in both vmcnt and lgkmcnt and may return out of order: every later wait then degenerates to
// vmcnt(0) lgkmcnt(0) and the software-pipelined prefetch of the next rounds is drained at every LDS add.
template <typename T> __device__ __forceinline__ T ldg_nt(const T* p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) T*)p);
}
template <typename T> __device__ __forceinline__ T ldg(const T* p) {
  return *((const __attribute__((address_space(1))) T*)p);
}
#define ROUNDS (NB / (NTHREADS * VEC))   // vector layout rounds (2)
#define SROUNDS (NB / NTHREADS)          // strided layout rounds (16)

template <typename VT> struct RawVals;
template <> struct RawVals<uint16_t> {
  v4u r;
  __device__ __forceinline__ void load(const uint16_t* p) { r = ldg_nt((const v4u*)p); }
  __device__ __forceinline__ void get(float* v) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = __uint_as_float(r[k] << 16);
      v[2 * k + 1] = __uint_as_float(r[k] & 0xffff0000u);
    }
  }
};
template <> struct RawVals<float> {
  v4f a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = ldg_nt((const v4f*)p);
    b = ldg_nt((const v4f*)(p + 4));
  }
  __device__ __forceinline__ void get(float* v) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[k] = a[k]; v[4 + k] = b[k]; }
  }
};
template <> struct RawVals<double> {
  v2d a[4];
  __device__ __forceinline__ void load(const double* p) {
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = ldg_nt((const v2d*)(p + 2 * k));
  }
  __device__ __forceinline__ void get(double* v) const {
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[2 * k] = a[k][0]; v[2 * k + 1] = a[k][1]; }
  }
};

__device__ __forceinline__ float val1(const uint16_t* p) {
  return __uint_as_float(((unsigned)ldg_nt(p)) << 16);
}
__device__ __forceinline__ float val1(const float* p) { return ldg_nt(p); }
__device__ __forceinline__ double val1(const double* p) { return ldg_nt(p); }

// Hot-table gather: lanes whose feature is in the LDS head read LDS; their global address collapses onto x[0]
// so that, whatever the compiler does with the predicated global load, they add no distinct cache lines.
template <typename XT, bool HOT>
__device__ __forceinline__ XT gather(const XT* __restrict__ x, const XT* hot, int hot_n, int j) {
  if (HOT) {
    const bool h = j < hot_n;
    const XT g = x[h ? 0 : j];
    return h ? hot[j] : g;
  }
  return x[j];
}

// ablation index transform (profiling builds only; abl == 0 in production)
__device__ __forceinline__ int abl_index(int abl, int j, int e) {
  if (abl & 1) return j & 255;            // 1 KB window: L1-resident gathers
  if (abl & 4) return j & 0xFFFF;         // 256 KB window: L2-resident random gathers
  if (abl & 8) return e & 0x3FFFF;        // perfectly coalesced gathers (consecutive entries)
  return j;
}

template <typename VT, typename XT, typename AT, bool SQ, bool STRIDED, bool HOT>
__device__ __forceinline__ double stream_products(const BlockDesc& d, const int* __restrict__ idx,
                                                  const VT* __restrict__ val, const XT* __restrict__ x,
                                                  const XT* hot, int hot_n, AT* prod, bool to_lds, int abl) {
  const int lo = d.nz_lo & ~(VEC - 1);
  const int hi = (d.nz_hi + VEC - 1) & ~(VEC - 1);
  double acc = 0.0;
  for (int base = lo; base < hi; base += NB) {
    if (STRIDED) {
      int ii[SROUNDS];
      AT v[SROUNDS];
#pragma unroll
      for (int r = 0; r < SROUNDS; ++r) {
        const int e = base + r * NTHREADS + threadIdx.x;
        ii[r] = e < hi ? ldg_nt(idx + e) : 0;
      }
#pragma unroll
      for (int r = 0; r < SROUNDS; ++r) {
        const int e = base + r * NTHREADS + threadIdx.x;
        v[r] = e < hi ? static_cast<AT>(val1(val + e)) : AT(0);
      }
      XT xv[SROUNDS];
#pragma unroll
      for (int r = 0; r < SROUNDS; ++r) {
        const int e = base + r * NTHREADS + threadIdx.x;
        const bool in = (e >= d.nz_lo) && (e < d.nz_hi);
        xv[r] = gather<XT, HOT>(x, hot, hot_n, abl_index(abl, in ? ii[r] : 0, e));
      }
      AT s = AT(0);
#pragma unroll
      for (int r = 0; r < SROUNDS; ++r) {
        const int e = base + r * NTHREADS + threadIdx.x;
        const bool in = (e >= d.nz_lo) && (e < d.nz_hi);
        const AT vv = SQ ? v[r] * v[r] : v[r];
        const AT p = in ? vv * static_cast<AT>(xv[r]) : AT(0);
        if (to_lds) {
          if (e < hi) prod[e - lo] = p;
        } else {
          s += p;
        }
      }
      if (!to_lds) acc += static_cast<double>(s);
    } else {
      v4i i0[ROUNDS], i1[ROUNDS];
      RawVals<VT> rv[ROUNDS];
#pragma unroll
      for (int r = 0; r < ROUNDS; ++r) {
        const int e = base + (r * NTHREADS + threadIdx.x) * VEC;
        if (e < hi) {
          i0[r] = ldg_nt((const v4i*)(idx + e));
          i1[r] = ldg_nt((const v4i*)(idx + e + 4));
          rv[r].load(val + e);
        }
      }
      XT xv[ROUNDS][8];
#pragma unroll
      for (int r = 0; r < ROUNDS; ++r) {
        const int e = base + (r * NTHREADS + threadIdx.x) * VEC;
        if (e < hi) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int ik = k < 4 ? i0[r][k] : i1[r][k - 4];
            const bool in = (e + k >= d.nz_lo) && (e + k < d.nz_hi);
            xv[r][k] = gather<XT, HOT>(x, hot, hot_n, abl_index(abl, in ? ik : 0, e + k));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < ROUNDS; ++r) {
        const int e = base + (r * NTHREADS + threadIdx.x) * VEC;
        if (e < hi) {
          AT v[8], p[8];
          rv[r].get(v);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const bool in = (e + k >= d.nz_lo) && (e + k < d.nz_hi);
            const AT vv = SQ ? v[k] * v[k] : v[k];
            p[k] = in ? vv * static_cast<AT>(xv[r][k]) : AT(0);
          }
          if (to_lds) {
            AT* q = prod + (e - lo);
#pragma unroll
            for (int k = 0; k < 8; ++k) q[k] = p[k];
          } else {
            AT s = AT(0);
#pragma unroll
            for (int k = 0; k < 8; ++k) s += p[k];
            acc += static_cast<double>(s);
          }
        }
      }
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
  double* z_out;      // MARGIN: z (double); VALUE_GRAD: margin cache; HV: direction margins (optional)
  int with_offset;    // MARGIN: add offset
  int abl;            // ablation bits (profiling only): 1 = gather from a 1 KB window, 2 = skip segmented reduce
  int hot_n;          // entries of x staged in LDS (features relabelled hottest-first), 0 = none
  // FWD_LS (margin-space line search, direction pass): z_out = zd (in: previous direction, out: new one),
  // z0 = cached margins (materialised here: z0 += tpend * zd_prev), first trial t0 -> (F, D) stats + coef
  double* z0; double t0; double tpend;
  // FWD_LS inputs: the margins z0 and the previous direction's margins are READ from here (the same buffers as
  // z0 / z_out for an in-place pass; the other buffer pair of the double-buffered margin cache for a speculative
  // pass, which must leave the current pair intact in case its line-search step is rejected)
  const double* z0_in; const double* zd_in;
};

// Per-row epilogue inputs, prefetched at block start (coalesced, latency hidden behind the stream phase)
template <typename XT, typename RT>
struct RowIn { RT y, off, wt; XT d; double z0, zd; };

template <typename XT, typename RT>
__device__ __forceinline__ RowIn<XT, RT> fwd_prefetch(const FwdArgs<XT, RT>& a, int s) {
  RowIn<XT, RT> r;
  r.y = RT(0); r.off = RT(0); r.wt = RT(0); r.d = XT(0); r.z0 = 0.0; r.zd = 0.0;
  if (a.mode == FWD_MARGIN) { if (a.with_offset) r.off = a.off[s]; }
  else if (a.mode == FWD_LS) { r.y = a.y[s]; r.wt = a.wt[s]; r.z0 = a.z0_in[s]; r.zd = a.zd_in[s]; }
  else if (a.mode == FWD_HV) { r.d = a.dzz[s]; }
  else { r.y = a.y[s]; r.off = a.off[s]; r.wt = a.wt[s]; }
  return r;
}

template <typename XT, typename RT>
__device__ __forceinline__ void fwd_finish(const FwdArgs<XT, RT>& a, int s, double sum, const RowIn<XT, RT>& r,
                                           double& F, double& S) {
  if (a.mode == FWD_MARGIN) {
    a.z_out[s] = sum + a.shift + static_cast<double>(r.off);
    return;
  }
  if (a.mode == FWD_LS) {
    const double zdn = sum + a.shift;                 // direction margin X d_eff + d_shift
    const double z0v = r.z0 + a.tpend * r.zd;         // accepted step of the previous line search
    a.z0[s] = z0v;
    a.z_out[s] = zdn;
    const double w = static_cast<double>(r.wt);
    double l, dl, d2;
    pointwise_loss(a.loss, z0v + a.t0 * zdn, static_cast<double>(r.y), l, dl, d2);
    a.coef[s] = static_cast<XT>(wx(w, dl));           // speculative: the transpose input if t0 is accepted
    F += wx(w, l);
    S += wx(w, dl * zdn);
    return;
  }
  if (a.mode == FWD_HV) {
    const double u = sum - a.shift;                   // margin change along the direction (X v_eff - v_eff.s)
    const double e = static_cast<double>(r.d) * u;
    a.coef[s] = static_cast<XT>(e);
    if (a.z_out) a.z_out[s] = u;                      // TRON: step margins accumulate sum_i alpha_i u_i
    S += e;
    return;
  }
  const double z = sum + a.shift + static_cast<double>(r.off);
  const double w = static_cast<double>(r.wt);
  double l, dl, d2;
  pointwise_loss(a.loss, z, static_cast<double>(r.y), l, dl, d2);
  if (a.mode == FWD_VALUE_GRAD) {
    a.coef[s] = static_cast<XT>(wx(w, dl));
    if (a.dzz) a.dzz[s] = static_cast<XT>(wx(w, d2));
    if (a.z_out) a.z_out[s] = z;  // margin cache for the margin-space line search (ls_eval_kernel)
    F += wx(w, l);
    S += wx(w, dl);
  } else {  // FWD_DZZ
    a.coef[s] = static_cast<XT>(wx(w, d2));
  }
}

#define HOT_BYTES 32768
#define MAXSEG_FWD 256            // forward (CSR) blocks hold <= 256 rows: one row per thread in the epilogue
#define SPT_FWD (MAXSEG_FWD / NTHREADS)
#define SPT_T (MAXSEG / NTHREADS)

// Shared-memory image of one block (kept in ONE struct so the kernels declare a single __shared__ object)
template <typename AT, typename XT, bool HOT, int MS>
struct BlockSmem {
  AT prod[NB + 2 * VEC];
  int segoff[MS + 1];
  double segsum[MS];
  double red[2 * NTHREADS / 64];
  XT hot[HOT ? HOT_BYTES / sizeof(XT) : 1];
};

// Phase A: segment sums from the LDS products into segsum[] (group size from the segment count).
template <typename AT, typename XT, bool HOT, int MS>
__device__ __forceinline__ void segment_sums(BlockSmem<AT, XT, HOT, MS>& sm, int nseg) {
  const int G = group_size(nseg);
  const int gid = threadIdx.x / G, gl = threadIdx.x % G, ngroups = NTHREADS / G;
  for (int base = 0; base < nseg; base += ngroups) {
    const int si = base + gid;
    double sum = 0.0;
    if (si < nseg) {
      const int b0 = sm.segoff[si], b1 = sm.segoff[si + 1];
      AT part = AT(0);
      for (int j = b0 + gl; j < b1; j += G) part += sm.prod[j];
      sum = static_cast<double>(part);
    }
    sum = group_reduce(sum, G);
    if (si < nseg && gl == 0) sm.segsum[si] = sum;
  }
}

// Persistent forward kernel: grid <= resident capacity; each workgroup (optionally) loads the LDS hot table once,
// then walks blocks b = blockIdx.x, +gridDim.x, ...  Per block: prefetch segment offsets (LDS) and per-row
// epilogue inputs (registers), stream + gather + products (LDS), segment sums, thread-per-row epilogue with
// coalesced row I/O, block (F, S) partials.
template <typename VT, typename XT, typename RT, typename AT, bool STRIDED, bool HOT>
__global__ __launch_bounds__(NTHREADS) void seg_fwd_kernel(
    const int* __restrict__ blk, int nblk, const int* __restrict__ seg_ptr, const int* __restrict__ idx,
    const VT* __restrict__ val, const XT* __restrict__ x, FwdArgs<XT, RT> a, double* __restrict__ stats,
    double* __restrict__ parts) {
  __shared__ __attribute__((aligned(16))) BlockSmem<AT, XT, HOT, MAXSEG_FWD> sm;
  const int hot_n = HOT ? a.hot_n : 0;
  if (HOT) {
    for (int i = threadIdx.x; i < hot_n; i += NTHREADS) sm.hot[i] = x[i];
    __syncthreads();
  }
  for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
    const BlockDesc d = load_desc(blk, b);
    if (d.part >= 0 || (a.abl & 2)) {
      double acc = stream_products<VT, XT, AT, false, STRIDED, HOT>(d, idx, val, x, sm.hot, hot_n, sm.prod, false,
                                                                    a.abl);
      double dummy = 0.0;
      block_sum2(acc, dummy, sm.red);
      if (threadIdx.x == 0 && d.part >= 0) parts[d.part] = acc;
      if (threadIdx.x == 0 && stats) { stats[2 * b] = (a.abl & 2) ? acc : 0.0; stats[2 * b + 1] = 0.0; }
      __syncthreads();
      continue;
    }
    const int lo = d.nz_lo & ~(VEC - 1);
    const int nseg = d.seg_hi - d.seg_lo;
    for (int i = threadIdx.x; i <= nseg; i += NTHREADS) sm.segoff[i] = seg_ptr[d.seg_lo + i] - lo;
    RowIn<XT, RT> pre[SPT_FWD];
#pragma unroll
    for (int k = 0; k < SPT_FWD; ++k) {
      const int si = threadIdx.x + k * NTHREADS;
      if (si < nseg) pre[k] = fwd_prefetch(a, d.seg_lo + si);
    }
    stream_products<VT, XT, AT, false, STRIDED, HOT>(d, idx, val, x, sm.hot, hot_n, sm.prod, true, a.abl);
    __syncthreads();
    segment_sums(sm, nseg);
    __syncthreads();
    double F = 0.0, S = 0.0;
#pragma unroll
    for (int k = 0; k < SPT_FWD; ++k) {
      const int si = threadIdx.x + k * NTHREADS;
      if (si < nseg) fwd_finish(a, d.seg_lo + si, sm.segsum[si], pre[k], F, S);
    }
    if (stats) {
      block_sum2(F, S, sm.red);
      if (threadIdx.x == 0) { stats[2 * b] = F; stats[2 * b + 1] = S; }
    }
    __syncthreads();  // LDS is rewritten by the next block
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
    const int s = long_seg[L];
    fwd_finish(a, s, sum, fwd_prefetch(a, s), F, S);
    if (long_stats) { long_stats[2 * L] = F; long_stats[2 * L + 1] = S; }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Transpose (row-chunked CSC): G[col] += sum_i val * x[row]   (SQ: val^2). The block's columns are a contiguous
// range, so the fp64 read-modify-write of G is prefetched at block start and written back coalesced.
template <typename VT, typename XT, typename AT, bool SQ, bool STRIDED>
__global__ __launch_bounds__(NTHREADS) void seg_t_kernel(const int* __restrict__ blk,
                                                         const int* __restrict__ seg_ptr,
                                                         const int* __restrict__ idx, const VT* __restrict__ val,
                                                         const XT* __restrict__ x, double* __restrict__ G,
                                                         double* __restrict__ parts, int abl) {
  __shared__ __attribute__((aligned(16))) BlockSmem<AT, XT, false, MAXSEG> sm;
  const BlockDesc d = load_desc(blk, blockIdx.x);
  if (d.part >= 0) {
    double acc = stream_products<VT, XT, AT, SQ, STRIDED, false>(d, idx, val, x, nullptr, 0, sm.prod, false, abl);
    double dummy = 0.0;
    block_sum2(acc, dummy, sm.red);
    if (threadIdx.x == 0) parts[d.part] = acc;
    return;
  }
  const int lo = d.nz_lo & ~(VEC - 1);
  const int nseg = d.seg_hi - d.seg_lo;
  for (int i = threadIdx.x; i <= nseg; i += NTHREADS) sm.segoff[i] = seg_ptr[d.seg_lo + i] - lo;
  double g0[SPT_T];
#pragma unroll
  for (int k = 0; k < SPT_T; ++k) {
    const int si = threadIdx.x + k * NTHREADS;
    g0[k] = si < nseg ? G[d.seg_lo + si] : 0.0;
  }
  stream_products<VT, XT, AT, SQ, STRIDED, false>(d, idx, val, x, nullptr, 0, sm.prod, true, abl);
  __syncthreads();
  segment_sums(sm, nseg);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SPT_T; ++k) {
    const int si = threadIdx.x + k * NTHREADS;
    if (si < nseg) G[d.seg_lo + si] = g0[k] + sm.segsum[si];
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
// TILED LAYOUT ("TL") — gather-coalesced kernels.
//
// Profiling the segmented-stream kernels showed them bound by the number of DISTINCT cache lines per gather
// instruction (~53 of 64 lanes hit different lines), not by HBM bytes. The tiled layout sorts each unit of work
// so that the lanes of one gather instruction hit neighbouring addresses, and accumulates through wave-private
// LDS (ds_add_f64) instead of segmented reductions:
//   forward  : ROW BLOCKS of <= 2^rbits rows; inside a block entries are sorted by (column, row) and packed as
//              (col << rbits) | local_row. Gathers x[col] walk the coefficient vector in order (hot columns, which
//              are relabelled to the lowest indices, collapse onto one or two lines per instruction).
//   transpose: COLUMN TILES of 2^cbits columns; inside a tile entries are sorted by (row, column) and packed as
//              (local_row << cbits) | (col & (2^cbits-1)). Gathers x[row] walk the per-row vector in order.
// Determinism: each wave owns a private LDS accumulator row and walks its entries in a fixed order, and the 4
// wave rows are summed in a fixed order; items of a column tile that is split across work-groups write fp64
// partial rows that a combine kernel adds IN ORDER. One assumption is MEASURED, not guaranteed by the ISA: when
// several lanes of ONE ds_add_f64 instruction hit the same LDS address, the LDS applies them in a fixed (lane)
// order. Every cross-instruction order is fixed by the program. Run-to-run bitwise equality is tested on each GPU
// run (tests/test_kernels_gpu.py: *bitwise* / determinism tests, torch.equal over repeated passes), and the
// fp64 results agree with the reference to ~1e-12 relative whatever the intra-instruction order.
// ============================================================================================================
#define TL_VEC 4                              // entries per lane per round (16-B pack loads)
#define TL_ROUND (64 * TL_VEC)                // entries per wave-round
#define TL_WAVES (NTHREADS / 64)
#define TL_MAXBITS 12                         // up to 4096 rows per forward block / columns per transpose tile

// Value quads: ``Raw`` is what one 4-entry load returns (kept as loaded so a prefetch does not force a wait),
// ``get`` converts to the arithmetic type at use.
template <typename VT> struct TLVals;
template <> struct TLVals<uint16_t> {
  typedef v2u Raw;
  static __device__ __forceinline__ Raw load(const uint16_t* p) { return ldg_nt((const v2u*)p); }
  static __device__ __forceinline__ void get(const Raw& u, float* v) {
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
};
template <> struct TLVals<float> {
  typedef v4f Raw;
  static __device__ __forceinline__ Raw load(const float* p) { return ldg_nt((const v4f*)p); }
  static __device__ __forceinline__ void get(const Raw& a, float* v) { v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; }
};
struct d4 { v2d a, b; };
template <> struct TLVals<double> {
  typedef d4 Raw;
  static __device__ __forceinline__ Raw load(const double* p) {
    d4 r;
    r.a = ldg_nt((const v2d*)p);
    r.b = ldg_nt((const v2d*)(p + 2));
    return r;
  }
  static __device__ __forceinline__ void get(const Raw& r, double* v) { v[0] = r.a[0]; v[1] = r.a[1]; v[2] = r.b[0]; v[3] = r.b[1]; }
};
template <typename VT> struct TLValT { typedef float T; };
template <> struct TLValT<double> { typedef double T; };

// block-wide sum of two doubles over NW waves; result valid in thread 0
template <int NW>
__device__ __forceinline__ void block_sum2_nw(double& a, double& b, double* sh /*[2*NW]*/) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) { sh[2 * w] = a; sh[2 * w + 1] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0; b = 0.0;
    for (int i = 0; i < NW; ++i) { a += sh[2 * i]; b += sh[2 * i + 1]; }
  }
}

// Stream entries [e_lo, e_hi) of one work unit: wave w walks a contiguous share of the 4-aligned window.
// For each entry: key = pack >> sbits (gather index), slot = pack & smask (LDS accumulator slot);
// acc[slot] += val (or val^2) * x[key]. U wave-rounds per iteration: all stream loads first, then all gathers,
// then the LDS accumulation (AT: float -> ds_add_f32, double -> ds_add_f64).
template <typename VT, typename XT, typename AT, bool SQ, int U, int NW>
__device__ __forceinline__ void tl_stream_p0(const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                          const XT* __restrict__ x, int e_lo, int e_hi, int sbits, AT* acc) {
  // Software-pipelined: the stream loads (pack + value quads) of round r + 1 are issued before the gathers and
  // LDS accumulation of round r, so the HBM latency of the stream overlaps with the gather latency.
  typedef typename TLValT<VT>::T LT;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t smask = (1u << sbits) - 1u;
  const int lo = e_lo & ~(TL_VEC - 1);
  const int nr = (e_hi - lo + TL_ROUND - 1) / TL_ROUND;
  const int r0 = (nr * w) / NW, r1 = (nr * (w + 1)) / NW;
  if (r0 >= r1) return;
  typedef typename TLVals<VT>::Raw Raw;
  // two prefetch slots (A: even rounds, B: odd rounds); the loop is unrolled by two so the slots stay in
  // registers (no dynamic indexing -> no scratch)
  v4u pkA, pkB;
  Raw vA, vB;
  auto load_round = [&](int r, v4u& pk, Raw& v) {
    const int e = lo + r * TL_ROUND + lane * TL_VEC;
    const int es = (r < r1 && e < e_hi) ? e : lo;  // out-of-range lanes re-read a valid quad; masked below
    pk = ldg_nt((const v4u*)(pack + es));
    v = TLVals<VT>::load(val + es);
  };
  auto process = [&](int r, v4u& pk_slot, Raw& v_slot) {
    const v4u pk = pk_slot;
    const Raw v_raw = v_slot;
    const int e = lo + r * TL_ROUND + lane * TL_VEC;
    bool in[TL_VEC];
    XT xv[TL_VEC];
#pragma unroll
    for (int k = 0; k < TL_VEC; ++k) {
      in[k] = (e + k >= e_lo) && (e + k < e_hi);
      xv[k] = ldg(x + (in[k] ? (pk[k] >> sbits) : 0u));  // unconditional: all four gathers in flight together
    }
    // refill this slot with round r + 2 AFTER issuing the gathers (vmcnt retires in issue order)
    if (r + 2 < r1) load_round(r + 2, pk_slot, v_slot);
    LT v[TL_VEC];
    TLVals<VT>::get(v_raw, v);
#pragma unroll
    for (int k = 0; k < TL_VEC; ++k) {
      if (in[k]) {
        const AT vv = SQ ? static_cast<AT>(v[k]) * static_cast<AT>(v[k]) : static_cast<AT>(v[k]);
        atomicAdd(&acc[pk[k] & smask], vv * static_cast<AT>(xv[k]));
      }
    }
  };
  load_round(r0, pkA, vA);
  if (r0 + 1 < r1) load_round(r0 + 1, pkB, vB);
  for (int r = r0; r < r1; r += 2) {
    process(r, pkA, vA);
    if (r + 1 < r1) process(r + 1, pkB, vB);
  }
}

template <typename VT, typename XT, typename AT, bool SQ, int U, int NW>
__device__ __forceinline__ void tl_stream_p1(const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                          const XT* __restrict__ x, int e_lo, int e_hi, int sbits, AT* acc) {
  // Three-stage software pipeline per wave (measured: removing the gathers halves the kernel time while
  // removing the LDS accumulation changes nothing, so the dependent stream-load -> gather -> accumulate chain
  // is latency bound):
  //   iteration r: issue gathers for round r+1 (its pack quad arrived one iteration ago), issue the stream loads
  //   of round r+2, then accumulate round r (its gathers were issued one iteration ago).
  // vmcnt retires in issue order, so the accumulation waits only for the gathers of round r while the six newer
  // loads stay in flight. Unrolled by two so the rotating slots stay in registers.
  typedef typename TLValT<VT>::T LT;
  typedef typename TLVals<VT>::Raw Raw;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t smask = (1u << sbits) - 1u;
  const int lo = e_lo & ~(TL_VEC - 1);
  const int nr = (e_hi - lo + TL_ROUND - 1) / TL_ROUND;
  const int r0 = (nr * w) / NW, r1 = (nr * (w + 1)) / NW;
  if (r0 >= r1) return;
  auto load_round = [&](int r, v4u& pk, Raw& v) {
    const int e = lo + r * TL_ROUND + lane * TL_VEC;
    const int es = (r < r1 && e < e_hi) ? e : lo;  // out-of-range lanes re-read a valid quad; masked below
    pk = ldg_nt((const v4u*)(pack + es));
    v = TLVals<VT>::load(val + es);
  };
  auto gather = [&](int r, const v4u& pk, XT* xv) {
    const int e = lo + r * TL_ROUND + lane * TL_VEC;
#pragma unroll
    for (int k = 0; k < TL_VEC; ++k) {
      const bool in = (r < r1) && (e + k >= e_lo) && (e + k < e_hi);
      xv[k] = ldg(x + (in ? (pk[k] >> sbits) : 0u));
    }
  };
  auto accumulate = [&](int r, const v4u& pk, const Raw& v_raw, const XT* xv) {
    const int e = lo + r * TL_ROUND + lane * TL_VEC;
    LT v[TL_VEC];
    TLVals<VT>::get(v_raw, v);
#pragma unroll
    for (int k = 0; k < TL_VEC; ++k) {
      if ((e + k >= e_lo) && (e + k < e_hi)) {
        const AT vv = SQ ? static_cast<AT>(v[k]) * static_cast<AT>(v[k]) : static_cast<AT>(v[k]);
        atomicAdd(&acc[pk[k] & smask], vv * static_cast<AT>(xv[k]));
      }
    }
  };
  // slots: A holds even rounds, B odd rounds
  v4u pkA, pkB;
  Raw vA, vB;
  XT xA[TL_VEC], xB[TL_VEC];
  load_round(r0, pkA, vA);
  load_round(r0 + 1, pkB, vB);
  gather(r0, pkA, xA);
  for (int r = r0; r < r1; r += 2) {
    // round r (slot A) accumulates; round r+1 (slot B) gathers; round r+2 streams into slot A
    gather(r + 1, pkB, xB);
    {
      const v4u pk = pkA;
      const Raw vv = vA;
      XT xc[TL_VEC];
#pragma unroll
      for (int k = 0; k < TL_VEC; ++k) xc[k] = xA[k];
      load_round(r + 2, pkA, vA);
      accumulate(r, pk, vv, xc);
    }
    if (r + 1 >= r1) break;
    // round r+1 (slot B) accumulates; round r+2 (slot A) gathers; round r+3 streams into slot B
    gather(r + 2, pkA, xA);
    {
      const v4u pk = pkB;
      const Raw vv = vB;
      XT xc[TL_VEC];
#pragma unroll
      for (int k = 0; k < TL_VEC; ++k) xc[k] = xB[k];
      load_round(r + 3, pkB, vB);
      accumulate(r + 1, pk, vv, xc);
    }
  }
}

// Two-slot prefetch like tl_stream_p0 with Q quads (4 * Q entries) per lane per round: Q = 2 doubles the
// loads and gathers each wave keeps in flight (memory-level parallelism per wave) at the cost of VGPRs.
template <typename VT, typename XT, typename AT, bool SQ, int NW, int Q>
__device__ __forceinline__ void tl_stream_wide(const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                            const XT* __restrict__ x, int e_lo, int e_hi, int sbits, AT* acc) {
  typedef typename TLValT<VT>::T LT;
  typedef typename TLVals<VT>::Raw Raw;
  constexpr int V = 4 * Q, ROUND = 64 * V;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t smask = (1u << sbits) - 1u;
  const int lo = e_lo & ~(TL_VEC - 1);
  const int nr = (e_hi - lo + ROUND - 1) / ROUND;
  const int r0 = (nr * w) / NW, r1 = (nr * (w + 1)) / NW;
  if (r0 >= r1) return;
  struct Slot { v4u pk[Q]; Raw v[Q]; };
  Slot A, B;
  auto load_round = [&](int r, Slot& sl) {
    const int e = lo + r * ROUND + lane * V;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int eq = e + 4 * q;
      const int es = (r < r1 && eq < e_hi) ? eq : lo;  // out-of-range quads re-read a valid one; masked below
      sl.pk[q] = ldg_nt((const v4u*)(pack + es));
      sl.v[q] = TLVals<VT>::load(val + es);
    }
  };
  auto process = [&](int r, Slot& sl) {
    v4u pk[Q];
    Raw vr[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) { pk[q] = sl.pk[q]; vr[q] = sl.v[q]; }
    const int e = lo + r * ROUND + lane * V;
    bool in[V];
    XT xv[V];
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = 4 * q + k;
        in[i] = (e + i >= e_lo) && (e + i < e_hi);
        xv[i] = ldg(x + (in[i] ? (pk[q][k] >> sbits) : 0u));
      }
    if (r + 2 < r1) load_round(r + 2, sl);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      LT v[4];
      TLVals<VT>::get(vr[q], v);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = 4 * q + k;
        if (in[i]) {
          const AT vv = SQ ? static_cast<AT>(v[k]) * static_cast<AT>(v[k]) : static_cast<AT>(v[k]);
          atomicAdd(&acc[pk[q][k] & smask], vv * static_cast<AT>(xv[i]));
        }
      }
    }
  };
  load_round(r0, A);
  if (r0 + 1 < r1) load_round(r0 + 1, B);
  for (int r = r0; r < r1; r += 2) {
    process(r, A);
    if (r + 1 < r1) process(r + 1, B);
  }
}

// Lane-interleaved stream (the "il" layout, ops/tiled.py): every work unit starts on a TL_ROUND boundary and is
// padded to whole rounds; inside a round of 256 sorted entries the quad of lane L holds the logical entries
// L, L+64, L+128, L+192. The 16-B stream loads stay fully coalesced, and gather k of a wave now reads 64
// CONSECUTIVE sorted entries (neighbouring columns in the forward, neighbouring rows in the transpose) instead of
// 64 entries spaced 4 apart, so each gather instruction touches ~4x fewer distinct cache lines in the sparse tail.
// No lower-bound masks (windows are round-aligned). Round-1 ablation (16M rows, bf16; profiles/
// kbench_il_ablation_16M.jsonl): without the coefficient gathers the streams ran at fwd 5.9 TB/s, transpose
// 4.6 TB/s; without the LDS adds nothing changed. A lane-run gather dedup (only run heads load, shuffle
// broadcast) measured 37 % slower (profiles/tl_dedup_ab_16M.txt) and was removed.

// Profiling ablations (experiment build only: -DPML_TL_EXPERIMENT, libpml_glm_abl.so, scripts/kbench.py
// --ablate): bit 1 -> register sums instead of the LDS atomics, bit 2 -> no coefficient gathers / key-window loads
// (x = 1), bit 4 -> fp32 products, bit 8 -> no wide-round gathers only, bit 16 -> no narrow key windows or
// permutes only, bit 32 -> no wide-round gathers of keys below ((abl >> 8) << 10) (the upper bound of serving the
// next tier of hot columns from an LDS table: those lanes skip the load), bit 64 -> the same but only for gather
// instructions whose 64 keys are all below the bound (the instruction is skipped; a wide section is sorted by key,
// so these are its hot prefix). The production build compiles TL_ABL to 0
// (no runtime checks).
#ifdef PML_TL_EXPERIMENT
__constant__ int c_tl_ablate = 0;
#define TL_ABL c_tl_ablate
#else
#define TL_ABL 0
#endif

// Ring-pipelined interleaved stream (P = 3: S = 2, D = 0; P = 5: S = 3, D = 1; P = 6: S = 5, D = 2): S rounds of
// stream in flight per wave and the gathers of round r + D issued before round r is accumulated.
// Code-generation rules that matter here (violating them serialised the loops: the waitcnt pass drained the
// whole queue, vmcnt(0), once per round — see README "Kernel pipelining"):
//  * the wave index is made wave-uniform (readfirstlane), so every loop bound and branch is scalar;
//  * every load is UNCONDITIONAL (past the end: a clamped re-read of the last round, never used), so the
//    outstanding-load sequence is the same on every path and every iteration;
//  * a ring of S + 1 register slots, refilled BEFORE the round in the oldest slot is processed, so a load never
//    targets a register that is still live (no loop-carried register copies, which force a wait on the load);
//  * no branch in the loop body: tail rounds (past r1) are processed with a select that adds an exact +0.0 (an
//    accumulator starting at +0.0 never holds -0.0, so the added zeros change no bits);
//  * a scheduling barrier keeps each step's loads ahead of its accumulation.
// Same entry order per wave for every (S, D): the result is bitwise identical across variants.
// WIDE-ROUND BASES (forward copies of shards whose column index does not fit 32 - rbits bits, ops/tiled.py):
// the pack holds the key relative to one int32 base per physical round, read with a scalar load when the round's
// streams are issued (``wbase``; a shard without bases passes a one-element zero table and stride 0, so the code
// path is the same). Masked lanes gather x[0].
__device__ const int g_zero_base[1] = {0};
typedef const __attribute__((address_space(4))) int* const_int_p;

template <typename VT, typename XT, typename AT, bool SQ, int NW, int S, int D>
__device__ __forceinline__ void tl_stream_ring(const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                               const XT* __restrict__ x, int e_lo, int e_hi, int sbits, AT* acc,
                                               const int* wbase) {
  constexpr int R = S + 1;
  static_assert(D < S && R % (D + 1) == 0, "gathers run ahead of loaded slots; the gather ring divides the slots");
  typedef typename TLValT<VT>::T LT;
  typedef typename TLVals<VT>::Raw Raw;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t smask = (1u << sbits) - 1u;
  const int nr = (e_hi - e_lo + TL_ROUND - 1) / TL_ROUND;
  const int r0 = (nr * w) / NW, r1 = (nr * (w + 1)) / NW;
  if (r0 >= r1) return;
  v4u pk[R];
  Raw vr[R];
  uint32_t bs[R];
  XT xg[D + 1][TL_VEC];
  const int ws = wbase ? 1 : 0;
  const const_int_p wb = (const_int_p)(wbase ? wbase : g_zero_base);
  const int rb0 = e_lo / TL_ROUND;                     // physical round index of the unit's first round
  auto load_round = [&](int r, v4u& p, Raw& v, uint32_t& b) {
    const int e = e_lo + min(r, r1 - 1) * TL_ROUND + lane * TL_VEC;
    p = ldg_nt((const v4u*)(pack + e));
    v = TLVals<VT>::load(val + e);
    b = (uint32_t)wb[ws * (rb0 + min(r, r1 - 1))];
  };
  const int abl = TL_ABL;
  AT regsum = AT(0);
  auto gather = [&](int r, const v4u& p, uint32_t b, XT* xv) {
    const int e = e_lo + r * TL_ROUND + lane;
#pragma unroll
    for (int k = 0; k < TL_VEC; ++k) {
      const uint32_t key = (e + 64 * k < e_hi) ? b + (p[k] >> sbits) : 0u;
      const bool hot = key < ((uint32_t)abl >> 8) << 10;
      if (abl & 10) xv[k] = XT(1);
      else if ((abl & 32) && hot) xv[k] = XT(1);                    // per lane (exec-masked load)
      else if ((abl & 64) && __ballot(!hot) == 0ull) xv[k] = XT(1);  // whole instruction skipped (all lanes hot)
      else xv[k] = ldg(x + key);
    }
  };
  // prologue in the steady state's issue order (loads of rounds r0 .. r0+S-1, then gathers of r0 .. r0+D-1), so
  // the outstanding-load sequence at the loop head is the same from the prologue and from the back edge
#pragma unroll
  for (int i = 0; i < S; ++i) {
    load_round(r0 + i, pk[i], vr[i], bs[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < D; ++i) {
    gather(r0 + i, pk[i], bs[i], xg[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int r = r0; r < r1; r += R) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rc = r + i;
      load_round(rc + S, pk[(i + S) % R], vr[(i + S) % R], bs[(i + S) % R]);   // slot of round rc - 1 (consumed)
      __builtin_amdgcn_sched_barrier(0);
      gather(rc + D, pk[(i + D) % R], bs[(i + D) % R], xg[(i + D) % (D + 1)]);   // gathers of round rc + D
      __builtin_amdgcn_sched_barrier(0);
      LT v[TL_VEC];
      TLVals<VT>::get(vr[i], v);
      const int e = e_lo + rc * TL_ROUND + lane;
#pragma unroll
      for (int k = 0; k < TL_VEC; ++k) {
        const bool in = (e + 64 * k < e_hi) && (rc < r1);
        const AT vv = SQ ? static_cast<AT>(v[k]) * static_cast<AT>(v[k]) : static_cast<AT>(v[k]);
        AT add;
        if (abl & 4) add = in ? static_cast<AT>(static_cast<float>(v[k]) * static_cast<float>(xg[i % (D + 1)][k]))
                              : AT(0);
        else add = in ? vv * static_cast<AT>(xg[i % (D + 1)][k]) : AT(0);  // select: no NaN from x
        if (abl & 1) regsum += add;
        else atomicAdd(&acc[in ? (pk[i][k] & smask) : 0u], add);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (abl & 1) atomicAdd(&acc[lane], regsum);
}

// NARROW rounds (ops/tiled.py, "narrow section" of a work unit): a round of 256 sorted entries whose gather keys
// span fewer than 64 values is stored with 16-bit packs ((key - base) << sbits | slot) plus one int32 base per
// round. Instead of four 64-lane gathers (the texture-address-bound part of the wide rounds: TA 80-94 % busy in
// profiles/pmc_tl_interleaved_4M.txt), the wave loads the round's whole key window x[base .. base+63] with ONE
// coalesced dword load and every lane picks its values with ds_bpermute (__shfl) from the window's lanes:
// 3 vector-memory instructions per round instead of 6, and 4 B/entry of stream instead of 6 (bf16).
// The layout builder guarantees base + 63 < len(x), so the window load is always in bounds. The bases are read
// with SCALAR loads (read-only data through the constant address space: s_load into SGPRs, counted in lgkmcnt,
// not in the vector-memory queue) one round ahead of the window load that needs them. Ring pipeline with S + 1
// slots under the code-generation rules of tl_stream_ring. Accumulation order per wave is fixed (deterministic).
template <typename T> __device__ __forceinline__ T lane_bcast(T v, int src) { return __shfl(v, src, 64); }

template <typename VT, typename XT, typename AT, bool SQ, int NW, int S = 2>
__device__ __forceinline__ void tl_stream_narrow(const uint16_t* __restrict__ npk, const VT* __restrict__ nvl,
                                                 const int* __restrict__ nbs, int n_lo, int n_hi, int sbits,
                                                 const XT* __restrict__ x, AT* acc) {
  constexpr int R = S + 1;
  typedef typename TLValT<VT>::T LT;
  typedef typename TLVals<VT>::Raw Raw;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nr = n_hi - n_lo;
  const int r0 = n_lo + (nr * w) / NW, r1 = n_lo + (nr * (w + 1)) / NW;
  if (r0 >= r1) return;
  const uint32_t smask = (1u << sbits) - 1u;
  const const_int_p bp = (const_int_p)nbs;
  v2u pks[R];
  Raw vs[R];
  XT xs[R];
  const int abl = TL_ABL;
  AT regsum = AT(0);
  auto issue = [&](int r, int base, v2u& pk, Raw& v, XT& xw) {
    const size_t e = (size_t)min(r, r1 - 1) * TL_ROUND + lane * TL_VEC;   // clamped re-read past the end
    pk = ldg_nt((const v2u*)(npk + e));
    v = TLVals<VT>::load(nvl + e);
    xw = (abl & 18) ? XT(1) : ldg(x + base + lane);
  };
#pragma unroll
  for (int i = 0; i < S; ++i) {
    issue(r0 + i, bp[min(r0 + i, r1 - 1)], pks[i], vs[i], xs[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  int nb = bp[min(r0 + S, r1 - 1)];
  for (int r = r0; r < r1; r += R) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rc = r + i;
      issue(rc + S, nb, pks[(i + S) % R], vs[(i + S) % R], xs[(i + S) % R]);   // slot of round rc - 1
      nb = bp[min(rc + S + 1, r1 - 1)];
      __builtin_amdgcn_sched_barrier(0);
      const bool live = rc < r1;          // tail rounds add an exact +0.0 (see tl_stream_ring)
      LT v[TL_VEC];
      TLVals<VT>::get(vs[i], v);
      const v2u pk = pks[i];
      const uint32_t p[TL_VEC] = {pk.x & 0xffffu, pk.x >> 16, pk.y & 0xffffu, pk.y >> 16};
#pragma unroll
      for (int k = 0; k < TL_VEC; ++k) {
        const XT xv = (abl & 16) ? xs[i] : lane_bcast(xs[i], (int)(p[k] >> sbits));
        const AT vv = SQ ? static_cast<AT>(v[k]) * static_cast<AT>(v[k]) : static_cast<AT>(v[k]);
        AT add;
        if (abl & 4) add = live ? static_cast<AT>(static_cast<float>(v[k]) * static_cast<float>(xv)) : AT(0);
        else add = live ? vv * static_cast<AT>(xv) : AT(0);
        if (abl & 1) regsum += add + AT(p[k] & smask);
        else atomicAdd(&acc[live ? (p[k] & smask) : 0u], add);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (abl & 1) atomicAdd(&acc[lane], regsum);
}

// pipeline variant: P = 0 two-slot stream prefetch; P = 1 three-stage (stream r+2 / gather r+1 / accumulate r);
// P = 2 two-slot, 8 entries per lane; P = 3 lane-interleaved layout (tl_stream_il)
template <typename VT, typename XT, typename AT, bool SQ, int U, int NW, int P>
__device__ __forceinline__ void tl_stream(const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                          const XT* __restrict__ x, int e_lo, int e_hi, int sbits, AT* acc,
                                          const int* wbase = nullptr) {
  // wide-round bases exist only in the interleaved layout (P >= 3); the builder never sets them otherwise
  if (P == 1) tl_stream_p1<VT, XT, AT, SQ, U, NW>(pack, val, x, e_lo, e_hi, sbits, acc);
  else if (P == 2) tl_stream_wide<VT, XT, AT, SQ, NW, 2>(pack, val, x, e_lo, e_hi, sbits, acc);
  else if (P == 3) tl_stream_ring<VT, XT, AT, SQ, NW, 2, 0>(pack, val, x, e_lo, e_hi, sbits, acc, wbase);
  else if (P == 5) tl_stream_ring<VT, XT, AT, SQ, NW, 3, 1>(pack, val, x, e_lo, e_hi, sbits, acc, wbase);
  else if (P == 6) tl_stream_ring<VT, XT, AT, SQ, NW, 5, 2>(pack, val, x, e_lo, e_hi, sbits, acc, wbase);
  else tl_stream_p0<VT, XT, AT, SQ, U, NW>(pack, val, x, e_lo, e_hi, sbits, acc);
}

// Narrow-section streams of one chunk (see tl_stream_narrow); n_lo == n_hi: the unit has no narrow rounds.
struct TLNarrow { const uint16_t* pack; const void* val; const int* base; const int* wbase; };

// Forward over row blocks. blk: 6 ints per block {row_lo, nrows, e_lo, e_hi, n_lo, n_hi} (chunk-local).
template <typename VT, typename XT, typename RT, typename AT, int MAXR, int U, int NW, int P>
__device__ __forceinline__ void tl_fwd_block(int b, int row_lo, int nrows, int e_lo, int e_hi, int n_lo, int n_hi,
                                             int rbits, const uint32_t* __restrict__ pack,
                                             const VT* __restrict__ val, const TLNarrow& nar,
                                             const XT* __restrict__ x, const FwdArgs<XT, RT>& a,
                                             double* __restrict__ stats, AT (*acc)[MAXR], double* red) {
  const int R = 1 << rbits;
  for (int i = threadIdx.x; i < R; i += NW * 64)
#pragma unroll
    for (int w = 0; w < NW; ++w) acc[w][i] = AT(0);
  __syncthreads();
  if (n_hi > n_lo)
    tl_stream_narrow<VT, XT, AT, false, NW, (P >= 5 ? 4 : 2)>(nar.pack, (const VT*)nar.val, nar.base, n_lo, n_hi,
                                                              rbits, x,
                                            acc[threadIdx.x >> 6]);
  tl_stream<VT, XT, AT, false, U, NW, P>(pack, val, x, e_lo, e_hi, rbits, acc[threadIdx.x >> 6], nar.wbase);
  __syncthreads();
  double F = 0.0, S = 0.0;
  for (int r = threadIdx.x; r < nrows; r += NW * 64) {
    double z = static_cast<double>(acc[0][r]);
#pragma unroll
    for (int w = 1; w < NW; ++w) z += static_cast<double>(acc[w][r]);
    const int s = row_lo + r;
    fwd_finish(a, s, z, fwd_prefetch(a, s), F, S);
  }
  if (stats) {
    block_sum2_nw<NW>(F, S, red);
    if (threadIdx.x == 0) { stats[2 * b] = F; stats[2 * b + 1] = S; }
  }
}

template <typename VT, typename XT, typename RT, typename AT, int MAXR, int U, int NW, int P>
__global__ __launch_bounds__(NW * 64) void tl_fwd_kernel(const int* __restrict__ blk, int rbits,
                                                          const uint32_t* __restrict__ pack,
                                                          const VT* __restrict__ val, TLNarrow nar,
                                                          const XT* __restrict__ x, FwdArgs<XT, RT> a,
                                                          double* __restrict__ stats,
                                                          const unsigned char* __restrict__ live) {
  __shared__ AT acc[NW][MAXR];
  __shared__ double red[2 * NW];
  const int b = blockIdx.x;
  if (live && !live[b]) return;
  const int* q = blk + 6 * b;
  tl_fwd_block<VT, XT, RT, AT, MAXR, U, NW, P>(b, q[0], q[1], q[2], q[3], q[4], q[5], rbits, pack, val, nar, x, a,
                                              stats, acc, red);
}

// All chunks of a shard in ONE launch (no per-chunk tails / launch gaps): block table of 8 ints
// {chunk, global row_lo, nrows, e_lo, e_hi, col_lo, n_lo, n_hi}; per-chunk stream pointers in device arrays
// (ptrs[6 * chunk + {0: pack, 1: val, 2: narrow pack, 3: narrow val, 4: narrow base, 5: wide-round bases or 0}]);
// row-data pointers in ``a``
// are shard-global; stats index = global block index.
template <typename VT, typename XT, typename RT, typename AT, int MAXR, int U, int NW, int P>
__global__ __launch_bounds__(NW * 64) void tl_fwd_multi_kernel(const int* __restrict__ blk, int rbits,
                                                                const unsigned long long* __restrict__ ptrs,
                                                                const XT* __restrict__ x, FwdArgs<XT, RT> a,
                                                                double* __restrict__ stats,
                                                                const unsigned char* __restrict__ live) {
  __shared__ AT acc[NW][MAXR];
  __shared__ double red[2 * NW];
  const int b = blockIdx.x;
  if (live && !live[b]) return;
  const int* q = blk + 8 * b;
  const unsigned long long* pc = ptrs + 6 * q[0];
  const TLNarrow nar = {(const uint16_t*)pc[2], (const void*)pc[3], (const int*)pc[4], (const int*)pc[5]};
  tl_fwd_block<VT, XT, RT, AT, MAXR, U, NW, P>(b, q[1], q[2], q[3], q[4], q[6], q[7], rbits, (const uint32_t*)pc[0],
                                              (const VT*)pc[1], nar, x + q[5], a, stats, acc, red);
}

// Transpose over column-tile items. items: 4 ints {tile, e_lo, e_hi, part}; part < 0: the item is its tile's
// only one -> G[tile cols] += sums directly; else the item's row of partial sums goes to parts[part * C ...].
template <typename VT, typename XT, typename AT, bool SQ, int MAXR, int U, int NW, int P>
__device__ __forceinline__ void tl_t_item(int tile, int e_lo, int e_hi, int part, int n_lo, int n_hi, int cbits,
                                          const uint32_t* __restrict__ pack, const VT* __restrict__ val,
                                          const TLNarrow& nar, const XT* __restrict__ x, double* __restrict__ G,
                                          int dim, double* __restrict__ parts, AT (*acc)[MAXR]) {
  const int C = 1 << cbits;
  for (int i = threadIdx.x; i < C; i += NW * 64)
#pragma unroll
    for (int w = 0; w < NW; ++w) acc[w][i] = AT(0);
  __syncthreads();
  if (n_hi > n_lo)
    tl_stream_narrow<VT, XT, AT, SQ, NW, (P >= 5 ? 4 : 2)>(nar.pack, (const VT*)nar.val, nar.base, n_lo, n_hi,
                                                           cbits, x,
                                         acc[threadIdx.x >> 6]);
  tl_stream<VT, XT, AT, SQ, U, NW, P>(pack, val, x, e_lo, e_hi, cbits, acc[threadIdx.x >> 6], nar.wbase);
  __syncthreads();
  const int c0 = tile << cbits;
  for (int c = threadIdx.x; c < C; c += NW * 64) {
    double s = static_cast<double>(acc[0][c]);
#pragma unroll
    for (int w = 1; w < NW; ++w) s += static_cast<double>(acc[w][c]);
    if (part < 0) {
      if (c0 + c < dim) G[c0 + c] += s;
    } else {
      parts[(size_t)part * C + c] = s;
    }
  }
}

template <typename VT, typename XT, typename AT, bool SQ, int MAXR, int U, int NW, int P>
__global__ __launch_bounds__(NW * 64) void tl_t_kernel(const int* __restrict__ items, int cbits,
                                                        const uint32_t* __restrict__ pack,
                                                        const VT* __restrict__ val, TLNarrow nar,
                                                        const XT* __restrict__ x, double* __restrict__ G, int dim,
                                                        double* __restrict__ parts,
                                                        const unsigned char* __restrict__ live) {
  __shared__ AT acc[NW][MAXR];
  if (live && !live[blockIdx.x]) return;
  const int* q = items + 6 * blockIdx.x;
  tl_t_item<VT, XT, AT, SQ, MAXR, U, NW, P>(q[0], q[1], q[2], q[3], q[4], q[5], cbits, pack, val, nar, x, G, dim,
                                            parts, acc);
}

// All row chunks of a shard in one launch. items: 8 ints {chunk, tile, e_lo, e_hi, part, row_base, n_lo, n_hi};
// a tile with a single item in the whole shard writes G directly, every other item writes a partial row that the
// shard-wide combine sums in (chunk, item) order — deterministic and race-free across chunks. Stream pointers as
// in tl_fwd_multi_kernel (6 per chunk).
template <typename VT, typename XT, typename AT, bool SQ, int MAXR, int U, int NW, int P>
__global__ __launch_bounds__(NW * 64) void tl_t_multi_kernel(const int* __restrict__ items, int cbits,
                                                              const unsigned long long* __restrict__ ptrs,
                                                              const XT* __restrict__ x, double* __restrict__ G,
                                                              int dim, double* __restrict__ parts,
                                                              const unsigned char* __restrict__ live,
                                                              const int* __restrict__ gate) {
  __shared__ AT acc[NW][MAXR];
  if (gate && *gate == 0) return;                       // gated pass (pml_set_gate): the step it serves was rejected
  if (live && !live[blockIdx.x]) return;
  const int* q = items + 8 * blockIdx.x;
  const unsigned long long* pc = ptrs + 6 * q[0];
  const TLNarrow nar = {(const uint16_t*)pc[2], (const void*)pc[3], (const int*)pc[4], (const int*)pc[5]};
  tl_t_item<VT, XT, AT, SQ, MAXR, U, NW, P>(q[1], q[2], q[3], q[4], q[6], q[7], cbits, (const uint32_t*)pc[0],
                                            (const VT*)pc[1], nar, x + q[5], G, dim, parts, acc);
}

// Combine the partial rows of split tiles, deterministically, in two levels (a hot tile can have hundreds of
// items: one work-group per tile would serialise its whole partial block):
//   level 1: unit u sums parts [cu[3u+1], cu[3u+2]) (<= TL_SEG consecutive items of one tile) -> l1[u * C + c]
//   level 2: tile t (blockIdx.x) sums its units [mt_ptr[t], mt_ptr[t+1]) in order, one column per thread
//            (blockIdx.y = column group), and adds into G.
// Fixed-order sum of rows [r0, r1) of ``src`` (rows of C doubles) at column c = blockIdx.y * 64 + lane: the 4 waves
// of the workgroup take contiguous quarters of the row range with 4 independent loads in flight per lane, and the
// quarters are added in order through LDS (result in wave 0). Deterministic: the split depends only on r1 - r0.
// (One thread per column looping over every row was latency bound: the hot tiles of a 125M-row shard hold ~200
// level-1 rows each, and only nmt x C / 256 workgroups ran — 1 ms per pass, profiles/bench_125M_timed_window.md.)
__device__ __forceinline__ double rows_sum64(const double* __restrict__ src, int C, int r0, int r1, int c,
                                             double* sh) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = r1 - r0;
  const int q0 = r0 + (n * w) / 4, q1 = r0 + (n * (w + 1)) / 4;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < C) {
    int r = q0;
    for (; r + 3 < q1; r += 4) {
      s0 += src[(size_t)r * C + c];
      s1 += src[(size_t)(r + 1) * C + c];
      s2 += src[(size_t)(r + 2) * C + c];
      s3 += src[(size_t)(r + 3) * C + c];
    }
    for (; r < q1; ++r) s0 += src[(size_t)r * C + c];
  }
  sh[w * 64 + lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  return (sh[lane] + sh[64 + lane]) + (sh[128 + lane] + sh[192 + lane]);
}

// level 1: unit u (rows p0..p1 of one split tile's item partial rows) -> l1 row u. Grid (ncu, C / 64), 256 threads.
__global__ __launch_bounds__(NTHREADS) void tl_t_combine1_kernel(const int* __restrict__ cu, int cbits,
                                                                 const double* __restrict__ parts,
                                                                 double* __restrict__ l1,
                                                                 const unsigned char* __restrict__ live_mt) {
  __shared__ double sh[NTHREADS];
  const int u = blockIdx.x;
  if (live_mt && !live_mt[cu[3 * u]]) return;           // whole workgroup
  const int C = 1 << cbits;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const double s = rows_sum64(parts, C, cu[3 * u + 1], cu[3 * u + 2], c, sh);
  if (threadIdx.x < 64 && c < C) l1[(size_t)u * C + c] = s;
}

// level 2: split tile t (its level-1 rows mt_ptr[t] .. mt_ptr[t+1]) -> G. Grid (nmt, C / 64), 256 threads.
__global__ __launch_bounds__(NTHREADS) void tl_t_combine2_kernel(const int* __restrict__ mt_tiles,
                                                                 const int* __restrict__ mt_ptr, int cbits,
                                                                 const double* __restrict__ l1,
                                                                 double* __restrict__ G, int dim,
                                                                 const unsigned char* __restrict__ live_mt) {
  __shared__ double sh[NTHREADS];
  const int t = blockIdx.x;
  if (live_mt && !live_mt[t]) return;                   // whole workgroup
  const int C = 1 << cbits;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const double s = rows_sum64(l1, C, mt_ptr[t], mt_ptr[t + 1], c, sh);
  if (threadIdx.x < 64 && c < C) {
    const int col = (mt_tiles[t] << cbits) + c;
    if (col < dim) G[col] += s;
  }
}

// ``il``: 1 = the streams are stored in the lane-interleaved layout (see tl_stream_il) -> pipeline P = 3.
// live: optional per-block flags (0 = skip the block: rows of converged entities in a block-diagonal problem)
struct TLFwdDesc { const int* blk; int nblk; int rbits; const uint32_t* pack; const void* val; int il; TLNarrow nar;
                  const unsigned char* live; };
// ptrs: 6 stream pointers per chunk (see tl_fwd_multi_kernel)
struct TLFwdMultiDesc { const int* blk; int nblk; int rbits; const unsigned long long* ptrs; int il;
                       const unsigned char* live; };
struct TLTDesc {
  const int* items; int nitems; int cbits; const uint32_t* pack; const void* val;
  const int* mt_tiles; const int* mt_ptr; int nmt; int dim;
  const int* cu; int ncu;     // level-1 combine units {tile, part_lo, part_hi}; mt_ptr indexes units
  int nparts_total;           // item partial rows (the level-1 rows follow them in the scratch buffer)
  int il;
  TLNarrow nar;
  const unsigned char* live;      // optional per-item flags (0 = skip) and per-split-tile flags for the combine
  const unsigned char* live_mt;
};
// Shard-wide transpose: items of every chunk (8 ints, see tl_t_multi_kernel) with per-chunk stream pointers.
struct TLTMultiDesc {
  const int* items; int nitems; int cbits; const unsigned long long* ptrs;
  const int* mt_tiles; const int* mt_ptr; int nmt; int dim;
  const int* cu; int ncu; int nparts_total; int il;
  const unsigned char* live;
  const unsigned char* live_mt;
};

// Runtime TL configuration: accumulator precision for bf16/f32 data (0 = fp32 LDS, 1 = fp64 LDS) and the number
// of waves per work-group (2 or 4: each wave owns an LDS accumulator row, so fewer waves = less LDS per WG = more
// resident WGs per CU). fp64 data always accumulates in fp64.
static int g_ablate = 0;      // profiling ablation bits (0 in production)
// FWD_LS arguments (set by pml_set_ls_args right before a direction pass; host-side, single stream)
static double* g_ls_z0 = nullptr;
static double g_ls_t0 = 0.0, g_ls_tpend = 0.0;
static const int* g_gate = nullptr;           // pml_set_gate: device flag read by the shard-wide transpose launch
static const double* g_ls_z0_in = nullptr;   // pml_set_ls_in: read-side buffers (null: the output buffers)
static const double* g_ls_zd_in = nullptr;
template <typename A>
static inline A& with_ls_in(A& a) {
  a.z0_in = g_ls_z0_in ? g_ls_z0_in : g_ls_z0;
  a.zd_in = g_ls_zd_in ? g_ls_zd_in : a.z_out;
  return a;
}
static int g_tl_acc64 = 1;   // measured on MI355X: ds_add_f64 accumulation is ~3x faster than ds_add_f32 here
static int g_tl_waves = 4;     // forward
static int g_tl_waves_t = 4;   // transpose
static int g_tl_pipe = 0;      // forward stream pipeline variant (see tl_stream)
static int g_tl_pipe_t = 0;    // transpose stream pipeline variant
static int g_rs_variant = 5;   // rs_tron variant: 0-2 rs_tron_kernel<V>; for n <= 32: 3 (5: one wave per workgroup
                                // for the LDS sizes, finer LDS occupancy granularity) rs_tron_dpp_kernel (L in registers
                                // for n <= 16; n in (20, 32]: packed lower triangle in LDS), 4 the same with L in
                                // LDS for every size, 6 one group-sum phase per CG step, 7 packed triangle for every
                                // n > 16; n > 32: 5 / 8 one problem per wave with permlane block rotation
                                // (scripts/rs_tron_bench.py, profiles/rs_tron_roofline.md)
static int g_tl_deep = 0;      // interleaved forward: 0 two-slot pipeline (P = 3), 1 deep S4/D1 (P = 5), 2 S6/D2 (P = 6)
static int g_tl_deep_t = 0;    // interleaved transpose: same

// Production builds compile only the production stream pipelines (interleaved layout: P = 3, plain: P = 0), the
// production wave counts (forward 2, transpose 4) and fp64 LDS accumulation; the A/B variants behind the runtime
// knobs (tl_pipe, tl_deep, tl_waves, tl_acc64) exist only in the experiment build (-DPML_TL_EXPERIMENT,
// ops/build.py build_experiment, loaded with PML_GLM_LIB), where the knobs select them.
#ifdef PML_TL_EXPERIMENT
#define TL_KNOB(x) (x)
#define TL_WAVES_F g_tl_waves
#define TL_WAVES_T g_tl_waves_t
#else
#define TL_KNOB(x) 0
#define TL_WAVES_F 2
#define TL_WAVES_T 4
#endif

template <typename VT, typename XT, typename RT, typename AT, int MAXR>
static void tl_fwd_launch(const TLFwdDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats, hipStream_t st) {
#define TLF(NW, P) hipLaunchKernelGGL((tl_fwd_kernel<VT, XT, RT, AT, MAXR, 2, NW, P>), dim3(c->nblk), dim3(NW * 64), 0, \
                                    st, c->blk, c->rbits, c->pack, (const VT*)c->val, c->nar, (const XT*)x, a, stats, \
                                    c->live)
  if (c->il) {
    if (TL_WAVES_F <= 2) { if (TL_KNOB(g_tl_deep) == 2) TLF(2, 6); else if (TL_KNOB(g_tl_deep)) TLF(2, 5); else TLF(2, 3); }
    else { if (TL_KNOB(g_tl_deep) == 2) TLF(4, 6); else if (TL_KNOB(g_tl_deep)) TLF(4, 5); else TLF(4, 3); }
  }
  else if (TL_WAVES_F == 2) { if (TL_KNOB(g_tl_pipe) == 1) TLF(2, 1); else TLF(2, 0); }
  else { if (TL_KNOB(g_tl_pipe) == 1) TLF(4, 1); else TLF(4, 0); }
#undef TLF
}

template <typename VT, typename XT, typename RT, typename AT, int MAXR>
static void tl_fwd_multi_launch(const TLFwdMultiDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats,
                                hipStream_t st) {
#define TLM(NW, P) hipLaunchKernelGGL((tl_fwd_multi_kernel<VT, XT, RT, AT, MAXR, 2, NW, P>), dim3(c->nblk), \
                                      dim3(NW * 64), 0, st, c->blk, c->rbits, c->ptrs, (const XT*)x, a, stats, \
                                      c->live)
  if (c->il) {
    if (TL_KNOB(g_tl_deep) == 2) { if (TL_WAVES_F == 2) TLM(2, 6); else TLM(4, 6); }
    else if (TL_KNOB(g_tl_deep)) { if (TL_WAVES_F == 2) TLM(2, 5); else TLM(4, 5); }
    else { if (TL_WAVES_F == 2) TLM(2, 3); else TLM(4, 3); }
  }
  else if (TL_WAVES_F == 2) { if (TL_KNOB(g_tl_pipe) == 2) TLM(2, 2); else TLM(2, 0); }
  else { if (TL_KNOB(g_tl_pipe) == 2) TLM(4, 2); else TLM(4, 0); }
#undef TLM
}

template <typename VT, typename XT, typename RT>
static int tl_fwd_multi_impl(const TLFwdMultiDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats,
                             hipStream_t st) {
  if (c->nblk <= 0) return 0;
  if (c->rbits < 1 || c->rbits > 11) return -22;
  const bool f64 = sizeof(XT) == 8 || !TL_KNOB(!g_tl_acc64);
  if (f64) {
    if (c->rbits <= 10) tl_fwd_multi_launch<VT, XT, RT, double, 1024>(c, x, a, stats, st);
    else tl_fwd_multi_launch<VT, XT, RT, double, 2048>(c, x, a, stats, st);
  } else {
    if (c->rbits <= 10) tl_fwd_multi_launch<VT, XT, RT, float, 1024>(c, x, a, stats, st);
    else tl_fwd_multi_launch<VT, XT, RT, float, 2048>(c, x, a, stats, st);
  }
  LAUNCH_CHECK();
  return 0;
}

template <typename VT, typename XT, typename RT>
static int tl_fwd_impl(const TLFwdDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats, hipStream_t st) {
  if (c->nblk <= 0) return 0;
  if (c->rbits < 1 || c->rbits > TL_MAXBITS) return -22;
  const bool f64 = sizeof(XT) == 8 || !TL_KNOB(!g_tl_acc64);
  if (f64) {
    if (c->rbits > 11) return -22;  // fp64 LDS: 4 waves x 2048 rows = 64 KB
    if (c->rbits <= 10) tl_fwd_launch<VT, XT, RT, double, 1024>(c, x, a, stats, st);
    else tl_fwd_launch<VT, XT, RT, double, 2048>(c, x, a, stats, st);
  } else if (c->rbits <= 10) {
    tl_fwd_launch<VT, XT, RT, float, 1024>(c, x, a, stats, st);
  } else if (c->rbits == 11) {
    tl_fwd_launch<VT, XT, RT, float, 2048>(c, x, a, stats, st);
  } else {
    tl_fwd_launch<VT, XT, RT, float, 4096>(c, x, a, stats, st);
  }
  LAUNCH_CHECK();
  return 0;
}

template <typename VT, typename XT, typename AT, bool SQ, int MAXR>
static void tl_t_launch(const TLTDesc* c, const void* x, double* G, double* parts, hipStream_t st) {
#define TLT(NW, P) hipLaunchKernelGGL((tl_t_kernel<VT, XT, AT, SQ, MAXR, 2, NW, P>), dim3(c->nitems), dim3(NW * 64), 0, \
                                    st, c->items, c->cbits, c->pack, (const VT*)c->val, c->nar, (const XT*)x, G, c->dim, \
                                    parts, c->live)
  if (c->il) {
    if (TL_WAVES_T == 2) { if (TL_KNOB(g_tl_deep_t) == 2) TLT(2, 6); else if (TL_KNOB(g_tl_deep_t)) TLT(2, 5); else TLT(2, 3); }
    else { if (TL_KNOB(g_tl_deep_t) == 2) TLT(4, 6); else if (TL_KNOB(g_tl_deep_t)) TLT(4, 5); else TLT(4, 3); }
  }
  else if (TL_WAVES_T == 2) { if (TL_KNOB(g_tl_pipe_t) == 1) TLT(2, 1); else TLT(2, 0); }
  else { if (TL_KNOB(g_tl_pipe_t) == 1) TLT(4, 1); else TLT(4, 0); }
#undef TLT
}

template <typename VT, typename XT, bool SQ>
static int tl_t_impl(const TLTDesc* c, const void* x, double* G, double* parts, hipStream_t st) {
  if (c->nitems <= 0) return 0;
  if (c->cbits < 1 || c->cbits > TL_MAXBITS) return -22;
  const bool f64 = sizeof(XT) == 8 || !TL_KNOB(!g_tl_acc64);
  if (f64) {
    if (c->cbits > 11) return -22;
    if (c->cbits <= 10) tl_t_launch<VT, XT, double, SQ, 1024>(c, x, G, parts, st);
    else tl_t_launch<VT, XT, double, SQ, 2048>(c, x, G, parts, st);
  } else if (c->cbits <= 10) {
    tl_t_launch<VT, XT, float, SQ, 1024>(c, x, G, parts, st);
  } else if (c->cbits == 11) {
    tl_t_launch<VT, XT, float, SQ, 2048>(c, x, G, parts, st);
  } else {
    tl_t_launch<VT, XT, float, SQ, 4096>(c, x, G, parts, st);
  }
  LAUNCH_CHECK();
  if (c->nmt > 0) {
    const int C = 1 << c->cbits;
    double* l1 = parts + (size_t)c->nparts_total * C;
    hipLaunchKernelGGL(tl_t_combine1_kernel, dim3(c->ncu, (C + 63) / 64), dim3(NTHREADS), 0, st, c->cu, c->cbits,
                       parts, l1, c->live_mt);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(tl_t_combine2_kernel, dim3(c->nmt, (C + 63) / 64), dim3(NTHREADS), 0, st,
                       c->mt_tiles, c->mt_ptr, c->cbits, l1, G, c->dim, c->live_mt);
    LAUNCH_CHECK();
  }
  return 0;
}

template <typename VT, typename XT, typename AT, bool SQ, int MAXR>
static void tl_t_multi_launch(const TLTMultiDesc* c, const void* x, double* G, double* parts, hipStream_t st) {
#define TLTM(NW, P) hipLaunchKernelGGL((tl_t_multi_kernel<VT, XT, AT, SQ, MAXR, 2, NW, P>), dim3(c->nitems), \
                                       dim3(NW * 64), 0, st, c->items, c->cbits, c->ptrs, (const XT*)x, G, \
                                       c->dim, parts, c->live, g_gate)
  if (c->il) {
    if (TL_WAVES_T == 2) { if (TL_KNOB(g_tl_deep_t) == 2) TLTM(2, 6); else if (TL_KNOB(g_tl_deep_t)) TLTM(2, 5); else TLTM(2, 3); }
    else { if (TL_KNOB(g_tl_deep_t) == 2) TLTM(4, 6); else if (TL_KNOB(g_tl_deep_t)) TLTM(4, 5); else TLTM(4, 3); }
  }
  else if (TL_WAVES_T == 2) { if (TL_KNOB(g_tl_pipe_t) == 2) TLTM(2, 2); else TLTM(2, 0); }
  else { if (TL_KNOB(g_tl_pipe_t) == 2) TLTM(4, 2); else TLTM(4, 0); }
#undef TLTM
}

template <typename VT, typename XT, bool SQ>
static int tl_t_multi_impl(const TLTMultiDesc* c, const void* x, double* G, double* parts, hipStream_t st) {
  if (c->nitems <= 0) return 0;
  if (c->cbits < 1 || c->cbits > 11) return -22;
  const bool f64 = sizeof(XT) == 8 || !TL_KNOB(!g_tl_acc64);
  if (f64) {
    if (c->cbits <= 10) tl_t_multi_launch<VT, XT, double, SQ, 1024>(c, x, G, parts, st);
    else tl_t_multi_launch<VT, XT, double, SQ, 2048>(c, x, G, parts, st);
  } else if (c->cbits <= 10) {
    tl_t_multi_launch<VT, XT, float, SQ, 1024>(c, x, G, parts, st);
  } else {
    tl_t_multi_launch<VT, XT, float, SQ, 2048>(c, x, G, parts, st);
  }
  LAUNCH_CHECK();
  if (c->nmt > 0) {
    const int C = 1 << c->cbits;
    double* l1 = parts + (size_t)c->nparts_total * C;
    hipLaunchKernelGGL(tl_t_combine1_kernel, dim3(c->ncu, (C + 63) / 64), dim3(NTHREADS), 0, st, c->cu, c->cbits,
                       parts, l1, c->live_mt);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(tl_t_combine2_kernel, dim3(c->nmt, (C + 63) / 64), dim3(NTHREADS), 0, st,
                       c->mt_tiles, c->mt_ptr, c->cbits, l1, G, c->dim, c->live_mt);
    LAUNCH_CHECK();
  }
  return 0;
}

// ============================================================================================================
// Segmented dot products for the block-diagonal random-effect solver: out[s] = sum_{i in [ptr[s], ptr[s+1])} f(a_i,
// b_i) with f = a*b (mode 0), a (mode 1), |a| (mode 2). One wave per segment, lane-strided fp64 partial sums
// combined by a fixed shuffle tree: deterministic, no atomics (replaces scatter-add with heavy contention).
// ============================================================================================================
__global__ __launch_bounds__(NTHREADS) void segdot_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                          int mode, const long long* __restrict__ ptr, int nseg,
                                                          double* __restrict__ out) {
  const int wv = (blockIdx.x * NTHREADS + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wv >= nseg) return;
  const long long lo = ptr[wv], hi = ptr[wv + 1];
  double s = 0.0;
  for (long long i = lo + lane; i < hi; i += 64) {
    const double x = a[i];
    s += mode == 0 ? x * b[i] : (mode == 1 ? x : fabs(x));
  }
  s = wave_sum(s);
  if (lane == 0) out[wv] = s;
}

// Long segments (a heavy-tail entity's 10^5..10^6 rows): one wave per segment serialises ~len / 64 dependent loads
// (a 1M-row segment: ~4.5 ms). segdot_long_kernel: the first `nseg_w` waves take the SHORT segments as above (long
// ones skip); the next waves take fixed chunks [w C, (w + 1) C) of the elements and sum the parts of the (at most
// two) LONG segments that overlap the chunk: head[w] for the segment holding the chunk's first element, tail[w] for
// one that starts inside the chunk. segdot_combine_kernel adds a long segment's parts in chunk order. Fixed
// partition, fixed order: deterministic (not bitwise equal to the one-wave form, whose lane strides differ).
#define SEGDOT_C 4096
__device__ __forceinline__ int seg_of(const long long* __restrict__ ptr, int nseg, long long i) {
  int lo = 0, hi = nseg - 1;                  // last s with ptr[s] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ptr[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ double seg_range_sum(const double* __restrict__ a, const double* __restrict__ b, int mode,
                                                long long lo, long long hi, int lane) {
  double s = 0.0;
  for (long long i = lo + lane; i < hi; i += 64) {
    const double x = a[i];
    s += mode == 0 ? x * b[i] : (mode == 1 ? x : fabs(x));
  }
  return wave_sum(s);
}

__global__ __launch_bounds__(NTHREADS) void segdot_long_kernel(const double* __restrict__ a,
                                                               const double* __restrict__ b, int mode,
                                                               const long long* __restrict__ ptr, int nseg,
                                                               int nseg_w, long long n, double* __restrict__ head,
                                                               double* __restrict__ tail, double* __restrict__ out) {
  const int wv = (blockIdx.x * NTHREADS + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wv < nseg_w) {
    if (wv >= nseg) return;
    const long long lo = ptr[wv], hi = ptr[wv + 1];
    if (hi - lo > SEGDOT_C) return;
    const double s = seg_range_sum(a, b, mode, lo, hi, lane);
    if (lane == 0) out[wv] = s;
    return;
  }
  const long long w = wv - nseg_w;
  const long long c0 = w * SEGDOT_C, c1 = c0 + SEGDOT_C < n ? c0 + SEGDOT_C : n;
  if (c0 >= n) return;
  const int s0 = seg_of(ptr, nseg, c0), s1 = seg_of(ptr, nseg, c1 - 1);
  double h = 0.0, t = 0.0;
  if (ptr[s0 + 1] - ptr[s0] > SEGDOT_C) h = seg_range_sum(a, b, mode, c0, ptr[s0 + 1] < c1 ? ptr[s0 + 1] : c1, lane);
  if (s1 != s0 && ptr[s1 + 1] - ptr[s1] > SEGDOT_C) t = seg_range_sum(a, b, mode, ptr[s1], c1, lane);
  if (lane == 0) { head[w] = h; tail[w] = t; }
}

__global__ __launch_bounds__(NTHREADS) void segdot_combine_kernel(const long long* __restrict__ ptr, int nseg,
                                                                  const double* __restrict__ head,
                                                                  const double* __restrict__ tail,
                                                                  double* __restrict__ out) {
  const int s = blockIdx.x * NTHREADS + threadIdx.x;
  if (s >= nseg) return;
  const long long lo = ptr[s], hi = ptr[s + 1];
  if (hi - lo <= SEGDOT_C) return;
  const long long w0 = lo / SEGDOT_C, w1 = (hi - 1) / SEGDOT_C;
  double acc = lo == w0 * SEGDOT_C ? head[w0] : tail[w0];
  for (long long w = w0 + 1; w <= w1; ++w) acc += head[w];
  out[s] = acc;
}

// Segment expansion: out[i] = src[e] for i in [ptr[e], ptr[e+1]) — per-entity scalars broadcast to the
// concatenated coefficient vector without reading an int64 index per element (one wave per segment).
template <typename T>
__global__ __launch_bounds__(NTHREADS) void seg_expand_kernel(const long long* __restrict__ ptr, int nseg,
                                                              const T* __restrict__ src, T* __restrict__ out) {
  const int e = (blockIdx.x * NTHREADS + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (e >= nseg) return;
  const long long lo = ptr[e], hi = ptr[e + 1];
  const T v = src[e];
  for (long long i = lo + lane; i < hi; i += 64) out[i] = v;
}

// ============================================================================================================
// Fused truncated-CG step of the block-diagonal random-effect TRON (photon-lib TRON.scala:279-339, one CG
// iteration for every entity at once). One wave per entity segment [ptr[e], ptr[e+1]) of the concatenated
// coefficient vector; per-entity scalars (rtr, delta, on-flag) live in device arrays. Per entity:
// Hd is the data part of the Hessian-vector product; the L2 term l2 * d is added on the fly (Hd + l2 d).
//   pass 1: dHd = d.Hd, std = step.d, sts = step.step, dtd = d.d           alpha = rtr / dHd
//   pass 2: |step + alpha d|^2 (explicit, as the reference)                hit = |trial| > delta, tau (boundary)
//   pass 3: step += (hit ? tau : alpha) d; r -= (hit ? tau : alpha) Hd; rnew = r.r
//   pass 4: (no hit) d = r + (rnew / rtr) d
// Replaces ~30 elementwise / gather / segmented-reduction launches per CG iteration with one; lane-strided
// partial sums + the fixed shuffle tree keep it deterministic and equal to segdot_kernel's dot products.
// ============================================================================================================
__global__ __launch_bounds__(NTHREADS) void seg_cg_step_kernel(const long long* __restrict__ ptr, int nseg,
                                                               double* __restrict__ step, double* __restrict__ r,
                                                               double* __restrict__ d, const double* __restrict__ Hd,
                                                               double* __restrict__ rtr, unsigned char* __restrict__ on,
                                                               const double* __restrict__ delta, double l2) {
  const int e = (blockIdx.x * NTHREADS + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (e >= nseg || !on[e]) return;
  const long long lo = ptr[e], hi = ptr[e + 1];
  double dhd = 0.0, std_ = 0.0, sts = 0.0, dtd = 0.0;
  for (long long i = lo + lane; i < hi; i += 64) {
    const double di = d[i], si = step[i];
    dhd += di * (Hd[i] + l2 * di);
    std_ += si * di;
    sts += si * si;
    dtd += di * di;
  }
  dhd = wave_sum(dhd); std_ = wave_sum(std_); sts = wave_sum(sts); dtd = wave_sum(dtd);
  const double rt = rtr[e];
  const double alpha = rt / (dhd == 0.0 ? 1.0 : dhd);
  double tn = 0.0;
  for (long long i = lo + lane; i < hi; i += 64) {
    const double t = step[i] + alpha * d[i];
    tn += t * t;
  }
  tn = wave_sum(tn);
  const double dl = delta[e];
  const bool hit = sqrt(tn > 0.0 ? tn : 0.0) > dl;
  double a = alpha;
  if (hit) {
    const double dsq = dl * dl;
    const double q = std_ * std_ + dtd * (dsq - sts);
    const double rad = sqrt(q > 0.0 ? q : 0.0);
    const double den1 = std_ + rad, den2 = dtd;
    a = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (den2 > 1e-300 ? den2 : 1e-300);
  }
  double rn = 0.0;
  for (long long i = lo + lane; i < hi; i += 64) {
    const double di = d[i];
    step[i] = step[i] + a * di;
    const double ri = r[i] - a * (Hd[i] + l2 * di);
    r[i] = ri;
    rn += ri * ri;
  }
  rn = wave_sum(rn);
  if (!hit) {
    const double beta = rn / (rt == 0.0 ? 1.0 : rt);
    for (long long i = lo + lane; i < hi; i += 64) d[i] = r[i] + beta * d[i];
  }
  if (lane == 0) {
    if (!hit) rtr[e] = rn;
    else on[e] = 0;
  }
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


// Runtime kernel configuration (set from Python): lane layout per direction, hot-table size, persistent grid.
static int g_fwd_strided = 0;
static int g_t_strided = 1;
static int g_hot_n = 0;          // requested LDS hot-table entries (clamped to HOT_BYTES / sizeof(XT))
static int g_fwd_grid = 256 * 4; // persistent forward grid (workgroups)

template <typename VT, typename XT, typename RT, typename AT, bool STRIDED, bool HOT>
static void launch_fwd(const SegChunkDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats, double* parts,
                       hipStream_t st) {
  const int grid = c->nblk < g_fwd_grid ? c->nblk : g_fwd_grid;
  hipLaunchKernelGGL((seg_fwd_kernel<VT, XT, RT, AT, STRIDED, HOT>), dim3(grid), dim3(NTHREADS), 0, st, c->blk,
                     c->nblk, c->seg_ptr, c->idx, (const VT*)c->val, (const XT*)x, a, stats, parts);
}

template <typename VT, typename XT, typename RT, typename AT>
static int fwd_impl(const SegChunkDesc* c, const void* x, FwdArgs<XT, RT> a, double* stats, double* long_stats,
                    double* parts, hipStream_t st) {
  const int max_hot = HOT_BYTES / (int)sizeof(XT);
  a.hot_n = g_hot_n < max_hot ? g_hot_n : max_hot;
  if (c->nblk > 0) {
    const bool hot = a.hot_n > 0;
    if (g_fwd_strided) {
      if (hot) launch_fwd<VT, XT, RT, AT, true, true>(c, x, a, stats, parts, st);
      else launch_fwd<VT, XT, RT, AT, true, false>(c, x, a, stats, parts, st);
    } else {
      if (hot) launch_fwd<VT, XT, RT, AT, false, true>(c, x, a, stats, parts, st);
      else launch_fwd<VT, XT, RT, AT, false, false>(c, x, a, stats, parts, st);
    }
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
    if (g_t_strided)
      hipLaunchKernelGGL((seg_t_kernel<VT, XT, AT, SQ, true>), dim3(c->nblk), dim3(NTHREADS), 0, st, c->blk,
                         c->seg_ptr, c->idx, (const VT*)c->val, (const XT*)x, G, parts, g_ablate);
    else
      hipLaunchKernelGGL((seg_t_kernel<VT, XT, AT, SQ, false>), dim3(c->nblk), dim3(NTHREADS), 0, st, c->blk,
                         c->seg_ptr, c->idx, (const VT*)c->val, (const XT*)x, G, parts, g_ablate);
    LAUNCH_CHECK();
  }
  if (c->nlong > 0) {
    hipLaunchKernelGGL(seg_t_long_kernel, dim3(c->nlong), dim3(64), 0, st, c->long_seg, c->long_ptr, parts, G);
    LAUNCH_CHECK();
  }
  return 0;
}

// ============================================================================================================
// Batched SMALL dense products for the row-space random-effect solve (optimization/row_space.py): a batch of
// B problems with n x n (n <= 64) fp64 design matrices. A wave owns per = floor(64 / n) CONSECUTIVE problems,
// i.e. one contiguous run of per * n^2 doubles: it is staged through LDS with coalesced loads (rows padded to
// n + 1 doubles: conflict-free row reads), then lane (g, i) = problem g's row / column i computes its dot
// product from LDS with x_j broadcast by shuffles. fp64 accumulation in a fixed order (deterministic).
// Measured on MI355X at 250K problems of 20 x 20: rocBLAS batched GEMM 0.63 ms, an L1-strided version of this
// kernel 1.0 ms (uncoalesced row reads thrash L1) — the staged form streams the blocks once.
// ============================================================================================================
__device__ __forceinline__ void stage_blocks(const double* __restrict__ A, long long b0, int count, int n,
                                             double* sA) {
  const int lane = threadIdx.x & 63;
  const int nn = n * n, np = n * (n + 1);
  const double* src = A + b0 * nn;
  const int tot = count * nn;
  for (int k = lane; k < tot; k += 64) {
    const int p = k / nn, rem = k - p * nn;
    const int i = rem / n, j = rem - i * n;
    sA[p * np + i * (n + 1) + j] = ldg_nt(src + k);
  }
}

__global__ __launch_bounds__(NTHREADS) void bgemv_kernel(int B, int n, const double* __restrict__ A,
                                                          const double* __restrict__ x, double* __restrict__ y,
                                                          int trans) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = 64 / n, np = n * (n + 1);
  double* sA = smem + w * per * np;
  const long long b0 = ((long long)blockIdx.x * (blockDim.x >> 6) + w) * per;
  if (b0 >= B) return;
  const int count = (int)min((long long)per, B - b0);
  stage_blocks(A, b0, count, n, sA);
  const int g = lane / n, i = lane - g * n;
  const bool on = g < count;
  const int base = lane - i;
  const double xi = on ? x[(b0 + g) * n + i] : 0.0;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const double* Ab = sA + (on ? g : 0) * np;
  double acc = 0.0;
  for (int j = 0; j < n; ++j) {
    const double xj = __shfl(xi, base + j, 64);
    acc = fma(trans ? Ab[j * (n + 1) + i] : Ab[i * (n + 1) + j], xj, acc);
  }
  if (on) y[(b0 + g) * n + i] = acc;
}

// 64 < n <= 192: one wave per problem straight from global memory (the block no longer fits a wave's LDS share);
// lane i owns rows i, i + 64, i + 128. x is staged in LDS (broadcast reads); A^T reads are coalesced over lanes,
// A reads walk each row (successive j hit the same cache lines: L1 hits).
// Batched triangular solves with the row-space Cholesky factors (optimization/row_space.py: beta = L^-1 z, the
// primal back-map's L^-T beta), replacing an explicitly formed inverse (O(n^3) per problem at setup and a second
// n x n matrix per problem in HBM). 64 / G problems per wave (G = pow2 >= n lanes each, one problem beyond 32):
// the lower triangles staged packed in LDS (coalesced reads; n <= 192: <= 148 KB), lane k of a problem holds entries
// k, k + 64, k + 128; n dependent steps, each: the pivot entry
// from its owner lane (readlane with one problem per wave, else a shuffle) times the diagonal's reciprocal (every
// lane: same value), then one fma per entry below (L y = x) or above (L^T y = x) the pivot.
__global__ __launch_bounds__(64) void btrsv_kernel(int B, int n, int G, const double* __restrict__ L,
                                                   const double* __restrict__ x, double* __restrict__ y, int trans) {
  // G = lanes per problem (pow2 >= n, <= 64): 64 / G problems per wave for n <= 32
  extern __shared__ double sl[];
  const int lane = threadIdx.x;
  const int P = 64 / G, q = lane / G, il = lane - q * G, tn = n * (n + 1) / 2;
  const long long b0 = (long long)blockIdx.x * P;
  if (b0 >= B) return;
  const int cnt = (int)min((long long)P, B - b0);
  // stage the lower triangles: BT_UNROLL loads in flight per lane before their LDS stores (one load at a time made
  // the staging a chain of dependent global-memory round trips: 0.67 ms for 18K problems of n = 64); entries above
  // the diagonal are not loaded
  const int nn = n * n, total = cnt * nn;
  const double* Lb = L + b0 * nn;
  constexpr int BT_UNROLL = 8;
  for (int t0 = 0; t0 < total; t0 += 64 * BT_UNROLL) {
    double v[BT_UNROLL];
    int dst[BT_UNROLL];
#pragma unroll
    for (int k = 0; k < BT_UNROLL; ++k) {
      const int t = t0 + 64 * k + lane;
      const int qq = t / nn, rem = t - qq * nn, r = rem / n, c = rem - r * n;
      const bool on = t < total && c <= r;
      dst[k] = on ? qq * tn + r * (r + 1) / 2 + c : -1;
      v[k] = on ? Lb[t] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < BT_UNROLL; ++k)
      if (dst[k] >= 0) sl[dst[k]] = v[k];
  }
  __syncthreads();
  // reciprocals of the diagonal, once: the n dependent steps then multiply instead of dividing
  double* rinv = sl + P * tn;
  for (int t = lane; t < cnt * n; t += 64) {
    const int qq = t / n, r = t - qq * n;
    rinv[qq * n + r] = 1.0 / sl[qq * tn + r * (r + 1) / 2 + r];
  }
  __syncthreads();
  const bool pon = q < cnt;
  const long long b = b0 + (pon ? q : 0);
  const double* sq = sl + (pon ? q : 0) * tn;
  const double* rq = rinv + (pon ? q : 0) * n;
  double v[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int k = il + 64 * s;
    v[s] = pon && k < n ? x[b * n + k] : 0.0;
  }
  for (int step = 0; step < n; ++step) {
    const int i = trans ? n - 1 - step : step;
    const int si = i >> 6;
    const double vi = si == 0 ? v[0] : (si == 1 ? v[1] : v[2]);
    double bi;
    if (P == 1) {       // one problem per wave: the pivot's lane is wave-uniform (readlane, no LDS crossbar)
      const long long u = __builtin_bit_cast(long long, vi);
      const int lo = __builtin_amdgcn_readlane((int)u, i & 63), hi = __builtin_amdgcn_readlane((int)(u >> 32), i & 63);
      bi = __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
    } else {
      bi = __shfl(vi, q * G + (i & 63), 64);
    }
    const double yi = bi * rq[i];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int k = il + 64 * s;
      if (k == i) {
        v[s] = yi;
      } else if (k < n && (trans ? k < i : k > i)) {
        const double lki = trans ? sq[i * (i + 1) / 2 + k] : sq[k * (k + 1) / 2 + i];
        v[s] = fma(-lki, yi, v[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int k = il + 64 * s;
    if (pon && k < n) y[b * n + k] = v[s];
  }
}

__global__ __launch_bounds__(256) void bgemv_wide_kernel(int B, int n, const double* __restrict__ A,
                                                         const double* __restrict__ x, double* __restrict__ y,
                                                         int trans) {
  __shared__ double sx[4][192];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long b = (long long)blockIdx.x * 4 + w;
  if (b >= B) return;
  const double* Ab = A + b * n * n;
  for (int j = lane; j < n; j += 64) sx[w][j] = x[b * n + j];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  double acc[3] = {0.0, 0.0, 0.0};
  for (int j = 0; j < n; ++j) {
    const double xj = sx[w][j];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int i = lane + 64 * r;
      if (i < n) acc[r] = fma(trans ? Ab[(long long)j * n + i] : Ab[(long long)i * n + j], xj, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int i = lane + 64 * r;
    if (i < n) y[b * n + i] = acc[r];
  }
}

// out = A^T (dw .* (A v)) + l2 v  (Hessian-vector product of the batched dense GLM, one read of each block)
__global__ __launch_bounds__(NTHREADS) void bhv_kernel(int B, int n, const double* __restrict__ A,
                                                        const double* __restrict__ dw, const double* __restrict__ v,
                                                        double l2, double* __restrict__ out) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = 64 / n, np = n * (n + 1);
  double* sA = smem + w * per * np;
  const long long b0 = ((long long)blockIdx.x * (blockDim.x >> 6) + w) * per;
  if (b0 >= B) return;
  const int count = (int)min((long long)per, B - b0);
  stage_blocks(A, b0, count, n, sA);
  const int g = lane / n, i = lane - g * n;
  const bool on = g < count;
  const int base = lane - i;
  const long long o = (b0 + (on ? g : 0)) * n + i;
  const double vi = on ? v[o] : 0.0;
  const double dwi = on ? dw[o] : 0.0;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const double* Ab = sA + (on ? g : 0) * np;
  double t = 0.0;
  for (int j = 0; j < n; ++j) t = fma(Ab[i * (n + 1) + j], __shfl(vi, base + j, 64), t);
  t *= dwi;
  double acc = 0.0;
  for (int r = 0; r < n; ++r) acc = fma(Ab[r * (n + 1) + i], __shfl(t, base + r, 64), acc);
  if (on) out[o] = acc + l2 * vi;
}

// ============================================================================================================
// Fused per-entity TRON for the row-space random-effect problems ("one workgroup per entity,
// dense tiles in LDS"). Each problem is a dense GLM with an n x n design matrix L (n <= 64, fp64): a lane group
// of G = pow2 >= n lanes owns one problem (lane i: data row i AND coefficient i), the block sits in LDS for the
// whole solve, and the complete trust-region Newton iteration — truncated CG with Hessian-vector products
// L^T (D (L d)), trust-region radius updates, accept / reject, Photon convergence tests — runs in registers.
// One HBM read of L per SOLVE instead of one per Hessian-vector product. Semantics follow batched_tron in
// optimization/batched.py (which follows TRON.scala:80-340): eta = (1e-4, .25, .75), sigma = (.25, .5, 4),
// delta0 = ||g0||, first-iteration delta = min(delta, ||step||), CG tolerance 0.1 ||g||, <= max_cg CG steps,
// <= max_fail consecutive rejections; reason codes 1 max-iter, 2 not-improving, 3 f-converged, 4 g-converged.
// Per-problem reductions are fixed-order butterflies inside the lane group: deterministic.
// ============================================================================================================
// Cross-lane moves of a double within a lane group, without the LDS crossbar where possible: DPP (quad
// permutations, row half-mirror / mirror: all inside 16 lanes) and ds_swizzle (xor 16 inside 32 lanes).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned int)lo);
}
template <int PAT>
__device__ __forceinline__ double swz_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)b, PAT);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), PAT);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned int)lo);
}

// V >= 1: the matrix-vector products read the vector from a per-problem LDS slot (one ds_write per product,
// then broadcast ds_reads) instead of two ds_bpermute shuffles per element, with two accumulators.
// V >= 2: group sums by DPP / swizzle steps instead of ds_bpermute butterflies (every step is symmetric, so all
// lanes of a group hold bitwise the same sum).
// L is lower triangular (Cholesky factor): only its n (n + 1) / 2 stored entries are staged, packed by rows
// (row i at i (i + 1) / 2), which halves the LDS per problem -- for the n > 32 classes (one problem per wave) LDS
// capped the occupancy at one wave per SIMD (33 KB per wave at n = 64). Full n x n rows are read from memory
// (coalesced) and the upper triangle dropped.
__device__ __forceinline__ void stage_lower(const double* __restrict__ A, long long b0, int count, int n,
                                            double* sA) {
  const int lane = threadIdx.x & 63;
  const int nn = n * n, np = n * (n + 1) / 2;
  const double* src = A + b0 * nn;
  const int tot = count * nn;
  for (int k = lane; k < tot; k += 64) {
    const int p = k / nn, rem = k - p * nn;
    const int i = rem / n, j = rem - i * n;
    const double v = ldg_nt(src + k);
    if (j <= i) sA[p * np + i * (i + 1) / 2 + j] = v;
  }
}

template <int V>
__global__ __launch_bounds__(NTHREADS) void rs_tron_kernel(
    int B, int n, int G, const double* __restrict__ Lm, const double* __restrict__ Y, const double* __restrict__ O,
    const double* __restrict__ WT, double* __restrict__ Beta, double* __restrict__ Fout, int* __restrict__ Iters,
    int* __restrict__ Reason, int loss, double l2, double tol, int max_iter, int max_fail, int max_cg,
    double* __restrict__ Zout) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = 64 / G, np = n * (n + 1) / 2;    // packed lower triangle per problem
  double* sA = smem + w * per * (np + (V >= 1 ? G : 0));
  double* sv = sA + per * np + (lane / G) * G;   // V = 1: this problem's vector slot
  const long long b0 = ((long long)blockIdx.x * (blockDim.x >> 6) + w) * per;
  if (b0 >= B) return;
  const int count = (int)min((long long)per, B - b0);
  stage_lower(Lm, b0, count, n, sA);
  const int g = lane / G, i = lane - g * G;
  const bool prob_on = g < count;
  const bool on = prob_on && i < n;
  const long long b = b0 + (prob_on ? g : 0);
  const long long o = b * n + (i < n ? i : 0);
  const double y = on ? Y[o] : 0.0, off = on ? O[o] : 0.0, wt = on ? WT[o] : 0.0;
  double W = on ? Beta[o] : 0.0;
  const int base = lane - i;
  const int ii = on ? i : 0;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const double* Lb = sA + (prob_on ? g : 0) * np;

  auto gsum = [&](double v) {
    if constexpr (V >= 2) {
      if (G >= 2) v += dpp_f64<0xB1>(v);      // quad_perm [1,0,3,2]
      if (G >= 4) v += dpp_f64<0x4E>(v);      // quad_perm [2,3,0,1]
      if (G >= 8) v += dpp_f64<0x141>(v);     // row_half_mirror
      if (G >= 16) v += dpp_f64<0x140>(v);    // row_mirror
      if (G >= 32) v += swz_f64<0x401F>(v);   // xor 16 within 32 lanes
      if (G >= 64) v += __shfl_xor(v, 32, 64);
      return v;
    } else {
      for (int s = G >> 1; s > 0; s >>= 1) v += __shfl_xor(v, s, 64);
      return v;
    }
  };
  auto put = [&](double v) {
    sv[i] = on ? v : 0.0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  };
  // packed lower triangle: L[r][c] (c <= r) at r (r + 1) / 2 + c; entries above the diagonal are 0 (reads past
  // a row's end land in the next row and are masked)
  auto mv = [&](double v) {  // (L v)_i
    const double* Lr = Lb + ii * (ii + 1) / 2;
    if constexpr (V >= 1) {
      put(v);
      double a0 = 0.0, a1 = 0.0;
      int j = 0;
      for (; j + 1 < n; j += 2) {
        a0 = fma(j <= ii ? Lr[j] : 0.0, sv[j], a0);
        a1 = fma(j + 1 <= ii ? Lr[j + 1] : 0.0, sv[j + 1], a1);
      }
      if (j < n) a0 = fma(j <= ii ? Lr[j] : 0.0, sv[j], a0);
      return on ? a0 + a1 : 0.0;
    } else {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc = fma(j <= ii ? Lr[j] : 0.0, __shfl(v, base + j, 64), acc);
      return on ? acc : 0.0;
    }
  };
  auto mvt = [&](double u) {  // (L^T u)_i
    if constexpr (V >= 1) {
      put(u);
      double a0 = 0.0, a1 = 0.0;
      int r = 0;
      for (; r + 1 < n; r += 2) {
        a0 = fma(r >= ii ? Lb[r * (r + 1) / 2 + ii] : 0.0, sv[r], a0);
        a1 = fma(r + 1 >= ii ? Lb[(r + 1) * (r + 2) / 2 + ii] : 0.0, sv[r + 1], a1);
      }
      if (r < n) a0 = fma(r >= ii ? Lb[r * (r + 1) / 2 + ii] : 0.0, sv[r], a0);
      return on ? a0 + a1 : 0.0;
    } else {
      double acc = 0.0;
      for (int r = 0; r < n; ++r) acc = fma(r >= ii ? Lb[r * (r + 1) / 2 + ii] : 0.0, __shfl(u, base + r, 64), acc);
      return on ? acc : 0.0;
    }
  };
  auto vg = [&](double v, double& f, double& gr, double& Dw) {
    const double z = mv(v) + off;
    double l, dl, d2;
    pointwise_loss(loss, z, y, l, dl, d2);
    if (!on) { l = 0.0; dl = 0.0; d2 = 0.0; }
    f = gsum(wt * l + 0.5 * l2 * v * v);
    gr = mvt(wt * dl) + l2 * v;
    Dw = wt * d2;
  };
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, s1 = 0.25, s2 = 0.5, s3 = 4.0;
  double f, gr, Dw;
  vg(W, f, gr, Dw);
  double f0z, g0n;
  if (gsum(W != 0.0 ? 1.0 : 0.0) == 0.0) {
    f0z = f;
    g0n = sqrt(gsum(gr * gr));
  } else {
    double f0, g0, D0;
    vg(0.0, f0, g0, D0);
    f0z = f0;
    g0n = sqrt(gsum(g0 * g0));
  }
  const double loss_tol = f0z * tol, grad_tol = g0n * tol;
  double delta = sqrt(gsum(gr * gr));
  int it = 0, fails = 0, reason = 0;
  bool active = prob_on;
  if (delta == 0.0) { reason = 4; active = false; }
  const int guard_max = max_iter * (max_fail + 1) + 5;
  for (int guard = 0; guard < guard_max; ++guard) {
    if (!__any(active)) break;
    // ---- truncated CG at W (Hessian weights Dw of the current iterate)
    double step = 0.0, r = -gr, d = r;
    double rtr = gsum(r * r);
    const double cg_tol = 0.1 * sqrt(gsum(gr * gr));
    bool cg_on = active;
    for (int k = 0; k < max_cg; ++k) {
      cg_on = cg_on && sqrt(rtr > 0.0 ? rtr : 0.0) > cg_tol;
      if (!__any(cg_on)) break;
      const double Hd = mvt(Dw * mv(d));
      const double Hl = Hd + l2 * d;
      const double dhd = gsum(d * Hl), std_ = gsum(step * d), sts = gsum(step * step), dtd = gsum(d * d);
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      const double tr = step + alpha * d;
      const double tn = gsum(tr * tr);
      const bool hit = sqrt(tn > 0.0 ? tn : 0.0) > delta;
      double a = alpha;
      if (hit) {
        const double dsq = delta * delta;
        const double q = std_ * std_ + dtd * (dsq - sts);
        const double rad = sqrt(q > 0.0 ? q : 0.0);
        const double den1 = std_ + rad;
        a = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300) : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
      }
      const double step_n = step + a * d;
      const double r_n = r - a * Hl;
      const double rn = gsum(r_n * r_n);
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
      if (cg_on) {
        step = step_n;
        r = r_n;
        if (!hit) { d = r_n + beta * d; rtr = rn; }
      }
      cg_on = cg_on && !hit;
    }
    // ---- trial point, trust-region update, acceptance
    const double Wn = W + step;
    const double gs = gsum(gr * step);
    const double pred = -0.5 * (gs - gsum(step * r));
    double fn, gn, Dn;
    vg(Wn, fn, gn, Dn);
    const double actual = f - fn;
    const double snorm = sqrt(gsum(step * step));
    if (active && it == 0) delta = fmin(delta, snorm);
    const double den = fn - f - gs;
    const double al = den <= 0.0 ? s3 : fmax(s1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(al, s1) * snorm, s2 * delta);
    else if (actual < eta1 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s2 * delta));
    else if (actual < eta2 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s3 * delta));
    else nd = fmax(delta, fmin(al * snorm, s3 * delta));
    if (active) delta = nd;
    const bool accept = active && actual > eta0 * pred;
    const double f_prev = f;
    if (accept) { W = Wn; f = fn; gr = gn; Dw = Dn; ++it; fails = 0; }
    else if (active) ++fails;
    const bool not_impr = active && !accept && fails >= max_fail;
    const double gnorm = sqrt(gsum(gr * gr));
    int rc = 0;
    if (accept && gnorm <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= max_iter) rc = 1;
    if (active && rc > 0) { reason = rc; active = false; }
  }
  if (on) Beta[o] = W;
  if (prob_on && i == 0) { Fout[b] = f; Iters[b] = it; Reason[b] = reason; }
  if (Zout != nullptr) {
    const double z = mv(W);       // the solution's margins L beta while L is still in LDS (no re-read of L)
    if (on) Zout[o] = z;
  }
}

// ============================================================================================================
// Variant 3 of the fused row-space TRON (n <= 32): problems of GL = 4 / 8 / 16 lanes (K <= 4 / 8 / else), K =
// the padded size (4, 8, 12, 16, 20, 24, 32), lane i holds vector entries i and (K > 16) i + 16.
// Measured on variant 2 (profiles/rs_tron_roofline.md): 7.4K VALU instructions per wave of 2 problems, only
// 20 % of them FMAs — the per-problem scalar work of truncated CG (divisions, square roots, trust-region
// selects, butterfly sums) runs once per WAVE, so it is paid per problem in proportion to 64 / lanes-per-problem.
// Here a wave holds 4 (K > 8), 8 or 16 problems, and every matrix-vector term is ONE instruction:
// v_fmac_f64_dpp with row_newbcast (DPP64) broadcasts the vector entry from lane k of the 16-lane row straight
// into the FMA (rs_dpp_blocks.h), with no LDS vector slot and no shuffles. L lives in registers for K <= 16 (row
// i and column i of L: 2K doubles per lane) and in LDS for K > 16 (zero-padded K x (K+1) rows per problem);
// triangular blocks of L above the diagonal are skipped. CG keeps ||step||^2 from the previous trial (the
// same sum), forms the boundary terms (step.d, d.d) only when some problem hits the trust region, and takes
// ||g||^2 = ||r0||^2: 3 group sums per CG step instead of 6. Same TRON semantics as rs_tron_kernel.
// ============================================================================================================
#include "rs_dpp_blocks.h"

// Build id (photon_ml_amd/ops/build.py: content hash of the sources + compile command, -DPML_BUILD_ID=...): the
// loaders compare it with the tree's sources and refuse a stale library.
#ifndef PML_BUILD_ID
#define PML_BUILD_ID "unstamped-build!"
#endif
__attribute__((used)) static const char pml_build_stamp[] = "PML_BUILD_ID=" PML_BUILD_ID;

// two independent group sums, stage by stage (ILP 2 on the DPP / add latency chain)
// Cross-row exchanges of a double for 64-lane problem groups (CDNA4 v_permlane16_swap / v_permlane32_swap, no LDS
// crossbar). pl_swap<16>(x) = (A, B) with A = [x0, x0, x2, x2], B = [x1, x1, x3, x3] per 16-lane row (rows 0-3);
// pl_swap<32>(x): A = [x0, x1, x0, x1], B = [x2, x3, x2, x3]. A + B is the xor-16 / xor-32 butterfly sum, in the
// same operand order on every lane (bitwise equal everywhere).
template <int D>
__device__ __forceinline__ void pl_swap(double x, double& A, double& B) {
  const long long b = __builtin_bit_cast(long long, x);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  unsigned alo, ahi, blo, bhi;
  if constexpr (D == 16) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    alo = rl[0]; blo = rl[1]; ahi = rh[0]; bhi = rh[1];
  } else {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    alo = rl[0]; blo = rl[1]; ahi = rh[0]; bhi = rh[1];
  }
  A = __builtin_bit_cast(double, ((unsigned long long)ahi << 32) | alo);
  B = __builtin_bit_cast(double, ((unsigned long long)bhi << 32) | blo);
}
template <int D>
__device__ __forceinline__ double pl_sum(double x) {
  double A, B;
  pl_swap<D>(x, A, B);
  return A + B;
}

template <int GL>
__device__ __forceinline__ void group_sum2(double& a, double& b) {
  a += dpp_f64<0xB1>(a); b += dpp_f64<0xB1>(b);
  a += dpp_f64<0x4E>(a); b += dpp_f64<0x4E>(b);
  if constexpr (GL >= 8) { a += dpp_f64<0x141>(a); b += dpp_f64<0x141>(b); }
  if constexpr (GL >= 16) { a += dpp_f64<0x140>(a); b += dpp_f64<0x140>(b); }
  if constexpr (GL >= 64) { a = pl_sum<16>(a); b = pl_sum<16>(b); a = pl_sum<32>(a); b = pl_sum<32>(b); }
}

// five independent group sums, stage by stage (ILP 5)
template <int GL>
__device__ __forceinline__ void group_sum5(double (&v)[5]) {
#pragma unroll
  for (int j = 0; j < 5; ++j) v[j] += dpp_f64<0xB1>(v[j]);
#pragma unroll
  for (int j = 0; j < 5; ++j) v[j] += dpp_f64<0x4E>(v[j]);
  if constexpr (GL >= 8) {
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] += dpp_f64<0x141>(v[j]);
  }
  if constexpr (GL >= 16) {
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] += dpp_f64<0x140>(v[j]);
  }
  if constexpr (GL >= 64) {
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] = pl_sum<16>(v[j]);
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] = pl_sum<32>(v[j]);
  }
}

template <int GL>
__device__ __forceinline__ double group_sum(double v) {
  v += dpp_f64<0xB1>(v);                       // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);                       // quad_perm [2,3,0,1]
  if constexpr (GL >= 8) v += dpp_f64<0x141>(v);   // row_half_mirror
  if constexpr (GL >= 16) v += dpp_f64<0x140>(v);  // row_mirror
  if constexpr (GL >= 64) { v = pl_sum<16>(v); v = pl_sum<32>(v); }
  return v;
}

// Masked reads of the packed triangle. SEL = false: a conditional read, which the compiler puts under an exec mask
// (SALU work; K = 32: 15.1 ms); SEL = true: an unconditional read + select (3 VALU per double, but fewer live
// registers: K = 24 fits 3 waves / SIMD with 6 spilled VGPRs instead of 22; 9.8 vs 10.3 ms)
__device__ __forceinline__ double tri_sel(double x, bool keep) {
  asm("" : "+v"(x));
  return keep ? x : 0.0;
}
#define tri_keep(x, keep) (Gm::SEL ? tri_sel((x), (keep)) : ((keep) ? (x) : 0.0))
#ifndef RS_SEL64
#define RS_SEL64 1
#endif
#ifndef RS_BLK64
#define RS_BLK64 1
#endif


template <int K, bool LREG, int WL = 2, bool TRI = false>
struct RsGeom {
  // K = 48 / 64 (variant 8): one problem per wave, lane i holds entry i (GL = 64)
  static constexpr int GL = K <= 4 ? 4 : (K <= 8 ? 8 : (K <= 32 ? 16 : 64));
  static constexpr int P = 64 / GL;                 // problems per wave
  static constexpr int R = GL == 64 ? 1 : (K + 15) / 16;   // vector entries per lane
  static constexpr bool REG = LREG && R == 1 && GL <= 16;  // L in registers (else LDS)
  static constexpr int K1 = K > 16 && GL == 16 ? K - 16 : 1;   // terms of the second column block
  static constexpr int SP = K + 1;                  // LDS row stride (doubles)
  // TRI (variant 7, K > 16): L packed as its lower triangle by rows, L[r][c] at r (r + 1) / 2 + c. The products
  // read whole 16-entry blocks and mask the entries above the diagonal; the last of them (column i + 16 at row
  // K - 1, i = 15) lies 32 - K + ... past the triangle, so the problem slot is padded to cover it
  static constexpr int TRI_N = GL == 64 ? 64 * 65 / 2   // GL = 64: unconditional reads of rows / columns < 64
                               : (K * (K + 1) / 2 > (K - 1) * K / 2 + 32) ? K * (K + 1) / 2 : (K - 1) * K / 2 + 32;
  // BLK (GL = 64): L as its lower-triangle 16 x 16 blocks (rows padded to 17 doubles: conflict-free row and column
  // reads); a product term whose block lies above the diagonal reads a stored block and takes a zero vector block
  // instead (the source is uniform over a DPP row) -- no masks at all
  static constexpr int NBK = (K + 15) / 16;
  // (200K problems: K = 48 9.51 -> 6.6 ms, 145 instead of 210 VGPRs; K = 64 12.3 -> 11.9 ms, 10 blocks = 21.8 KB
  // per wave; profiles/rs_tron_roofline.md)
  static constexpr bool BLK = GL == 64 && RS_BLK64;
  static constexpr int PS0 = BLK ? NBK * (NBK + 1) / 2 * 272 : (TRI && (R == 2 || GL == 64)) ? TRI_N : K * SP;
  static constexpr bool SEL = K == 24 || (GL == 64 && RS_SEL64);   // masked reads: select (else exec-masked; tri_keep)
  // problem stride = 16 mod 32 doubles (measured: dropping the pad to fit 12 one-wave workgroups per CU at K = 20
  // gains nothing over variant 5, 7.66 vs 7.69 ms, and loses 3 % at K = 24)
  static constexpr int PS = PS0 + (((16 - PS0 % 32) % 32) + 32) % 32;
  static constexpr int WPB = REG ? 4 : WL;          // waves per workgroup (LDS sizes: WL, see variant 5)
};

// MS (variant 6): ONE group-sum phase per CG step — d.Hd, step.d, d.d, r.Hd and Hd.Hd summed together (five
// independent DPP chains), the trial norm and the new residual norm by algebra:
//   ||step + a d||^2 = ||step||^2 + 2 a step.d + a^2 d.d,   ||r - a Hd||^2 = r.r - 2 a r.Hd + a^2 Hd.Hd
// (clamped at 0). The baseline variant pays a serial sum for d.Hd, then one for the two norms, and a third when a
// problem hits the trust region.
// occupancy asked of the register allocator (waves per SIMD): the packed-triangle K = 20 build lands 1 VGPR over
// the 3-wave budget of 168 without it
#ifndef RS_WPE20
#define RS_WPE20 3
#endif
#ifndef RS_WPE24
#define RS_WPE24 3
#endif
#ifndef RS_WPE32
#define RS_WPE32 1
#endif
#ifndef RS_WPE48
#define RS_WPE48 1
#endif
#ifndef RS_WPE64
#define RS_WPE64 1
#endif
template <int K, bool TRI>
constexpr int rs_dpp_wpe() {
  return !TRI ? 1 : K == 20 ? RS_WPE20 : K == 24 ? RS_WPE24 : K == 32 ? RS_WPE32 : K == 48 ? RS_WPE48
                  : K == 64 ? RS_WPE64 : 1;
}

template <int K, bool LREG, int WL, bool MS = false, bool TRI = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(rs_dpp_wpe<K, TRI>()))) void rs_tron_dpp_kernel(
    int B, int n, const double* __restrict__ Lm, const double* __restrict__ Y, const double* __restrict__ O,
    const double* __restrict__ WT, double* __restrict__ Beta, double* __restrict__ Fout, int* __restrict__ Iters,
    int* __restrict__ Reason, int loss, double l2, double tol, int max_iter, int max_fail, int max_cg,
    const int* __restrict__ order, double* __restrict__ Zout) {
  using Gm = RsGeom<K, LREG, WL, TRI>;
  constexpr int GL = Gm::GL, P = Gm::P, R = Gm::R, K1 = Gm::K1, SP = Gm::SP, PS = Gm::PS;
  constexpr bool PK = TRI && (R == 2 || GL == 64);   // packed lower triangle in LDS
  extern __shared__ double smem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane / GL, i = lane % GL;
  const long long b0 = ((long long)blockIdx.x * Gm::WPB + w) * P;
  if (b0 >= B) return;
  const bool prob_on = b0 + q < B;
  // order (optional): the wave's problems are order[b0 .. b0 + P) -- problems of similar difficulty share a wave
  // (a wave runs until its slowest problem finishes); results go to the problems' own slots
  auto prob = [&](long long j) -> long long { return order ? (long long)order[j] : j; };
  const long long b = prob(prob_on ? b0 + q : b0);
  const long long nn = (long long)n * n;
  bool on[R];
  long long o[R];
  double W[R];
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const int e = i + 16 * s;
    on[s] = prob_on && e < n;
    o[s] = b * n + (e < n ? e : 0);
    W[s] = on[s] ? Beta[o[s]] : 0.0;
  }
  // ---- L: registers (row i and column i) or LDS (zero-padded, this wave's P problems)
  double Lr[Gm::REG ? K : 1], Lc[Gm::REG ? K : 1];
  int lq = 0;                                   // this problem's LDS base (doubles)
  if constexpr (Gm::REG) {
    const double* Lb = Lm + b * nn;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool ok = prob_on && i < n && k < n;
      Lr[k] = ok ? Lb[(long long)i * n + k] : 0.0;
      Lc[k] = ok ? Lb[(long long)k * n + i] : 0.0;
    }
  } else if constexpr (Gm::BLK) {
    // one problem per wave: zero the slot (upper halves of the diagonal blocks, row pads), then the lower triangle
    // into its blocks
    const int wb = w * PS;
    for (int idx = lane; idx < PS; idx += 64) smem[wb + idx] = 0.0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (prob_on) {
      const double* Lb = Lm + b * nn;
      for (int idx = lane; idx < n * n; idx += 64) {
        const int r = idx / n, c = idx - r * n;
        if (c <= r) smem[wb + ((r >> 4) * ((r >> 4) + 1) / 2 + (c >> 4)) * 272 + (r & 15) * 17 + (c & 15)] = Lb[idx];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    lq = wb;
  } else if constexpr (PK) {
    // this wave's P problems, read row-major (coalesced) and stored packed; slot tails (the masked over-reads
    // past the triangle) zero
    const int wb = w * P * PS;
    for (int idx = lane; idx < P * (PS - Gm::TRI_N + K * K); idx += 64) {
      const int qq = idx / (PS - Gm::TRI_N + K * K), rem = idx - qq * (PS - Gm::TRI_N + K * K);
      if (rem < K * K) {
        const int r = rem / K, c = rem - r * K;
        if (c <= r) {
          double v = 0.0;
          if (b0 + qq < B && r < n && c < n) v = Lm[prob(b0 + qq) * nn + (long long)r * n + c];
          smem[wb + qq * PS + r * (r + 1) / 2 + c] = v;
        }
      } else {
        smem[wb + qq * PS + K * (K + 1) / 2 + (rem - K * K)] = 0.0;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    lq = wb + q * PS;
  } else {
    const int wb = w * P * PS;
    for (int idx = lane; idx < P * PS; idx += 64) {
      const int qq = idx / PS, rem = idx - qq * PS, r = rem / SP, c = rem - r * SP;
      double v = 0.0;
      if (b0 + qq < B && r < n && c < n) v = Lm[prob(b0 + qq) * nn + (long long)r * n + c];
      smem[wb + idx] = v;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    lq = wb + q * PS;
  }
  // sum_k m[k] * (entry k of the lane's problem vector), L in registers
  auto reg_mv = [&](double v, const double (&m)[R == 1 ? K : 1]) {
    if constexpr (R != 1 || GL > 16) {
      return 0.0;
    } else if constexpr (GL == 16) {
      double a0 = 0.0, a1 = 0.0;
      bcf<16, K>(a0, a1, v, m);
      return a0 + a1;
    } else {
      double acc[16 / GL];
#pragma unroll
      for (int g = 0; g < 16 / GL; ++g) acc[g] = 0.0;
      bcg<GL, K>(acc, v, m);
      const int mine = (lane & 15) / GL;
      double r = acc[0];
#pragma unroll
      for (int g = 1; g < 16 / GL; ++g) r = mine == g ? acc[g] : r;
      return r;
    }
  };
  // (L v) and (L^T u) for the lane's entries; entries >= n are 0 on input and on output
  auto mv = [&](const double (&v)[R], double (&out)[R]) {
    if constexpr (Gm::REG) {
      out[0] = on[0] ? reg_mv(v[0], Lr) : 0.0;
    } else if constexpr (R == 1 && GL <= 16) {
      double m[K];
      int base = lq + i * SP;
      asm volatile("" : "+v"(base));   // re-read L from LDS in every product (no hoisting into registers)
#pragma unroll
      for (int k = 0; k < K; ++k) m[k] = smem[base + k];
      out[0] = on[0] ? reg_mv(v[0], m) : 0.0;
    } else if constexpr (GL == 64) {
      // one problem per wave, lane i = 16 a + ii holds entry i. Column block b = a ^ s of the vector reaches row a
      // through a permlane swap (s = 1: xor 16, s = 2: xor 32, s = 3: both), then row_newbcast:k broadcasts its
      // entry k into the FMA. BLK (K = 48): rows of the stored 16 x 16 blocks, above-diagonal terms multiply a
      // zero vector block; otherwise rows of the packed triangle with blocks above the diagonal (b > a) and entries
      // k > ii of the diagonal block masked (tri_keep: select)
      const int a = i >> 4, ii = i & 15;
      double S[4], A, Bv;
      S[0] = v[0];
      pl_swap<16>(v[0], A, Bv);
      S[1] = (a & 1) ? A : Bv;
      pl_swap<32>(v[0], A, Bv);
      S[2] = (a & 2) ? A : Bv;
      pl_swap<32>(S[1], A, Bv);
      S[3] = (a & 2) ? A : Bv;
      double a0 = 0.0, a1 = 0.0;
      if constexpr (Gm::BLK) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int bb = a ^ s;
          const bool lower = a < Gm::NBK && bb <= a;
          int base = lq + (lower ? a * (a + 1) / 2 + bb : 0) * 272 + ii * 17;
          asm volatile("" : "+v"(base));
          double m[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) m[k] = smem[base + k];
          bcf<16, 16>(a0, a1, lower ? S[s] : 0.0, m);
        }
        out[0] = on[0] ? a0 + a1 : 0.0;
        return;
      }
      int rb = lq + i * (i + 1) / 2;
      asm volatile("" : "+v"(rb));
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int cb = rb + 16 * (a ^ s);
        const bool below = (a ^ s) < a && i < K;
        double m[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) m[k] = tri_keep(smem[cb + k], s == 0 ? (k <= ii && i < K) : below);
        bcf<16, 16>(a0, a1, S[s], m);
      }
      out[0] = on[0] ? a0 + a1 : 0.0;
    } else if constexpr (PK) {
      // rows i and i + 16 of the packed triangle; entries above the diagonal (k > i in the diagonal blocks) read
      // the next row and are masked to 0 (the same products as the padded layout's stored zeros)
      double m[16], m1[K1];
      const int i1 = min(i + 16, K - 1);
      int b0i = lq + i * (i + 1) / 2, b1i = lq + i1 * (i1 + 1) / 2;
      asm volatile("" : "+v"(b0i), "+v"(b1i));
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = tri_keep(smem[b0i + k], k <= i);
      double a0 = 0.0, a1 = 0.0;
      bcf<16, 16>(a0, a1, v[0], m);
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = smem[b1i + k];
#pragma unroll
      for (int k = 0; k < K1; ++k) m1[k] = tri_keep(smem[b1i + 16 + k], k <= i);
      double c0 = 0.0, c1 = 0.0;
      bcf<16, 16>(c0, c1, v[0], m);
      bcf<16, K1>(c0, c1, v[1], m1);
      out[0] = on[0] ? a0 + a1 : 0.0;
      out[1] = on[1] ? c0 + c1 : 0.0;
    } else {
      double m[16], m1[K1];
      // re-read L from LDS in every product: laundering the (integer) base keeps the compiler from hoisting
      // all 2K^2/16 values per lane out of the CG loop into (spilled) registers
      int b0i = lq + i * SP, b1i = lq + min(i + 16, K - 1) * SP;
      asm volatile("" : "+v"(b0i), "+v"(b1i));
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = smem[b0i + k];
      double a0 = 0.0, a1 = 0.0;
      bcf<16, 16>(a0, a1, v[0], m);
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = smem[b1i + k];
#pragma unroll
      for (int k = 0; k < K1; ++k) m1[k] = smem[b1i + 16 + k];
      double c0 = 0.0, c1 = 0.0;
      bcf<16, 16>(c0, c1, v[0], m);
      bcf<16, K1>(c0, c1, v[1], m1);
      out[0] = on[0] ? a0 + a1 : 0.0;
      out[1] = on[1] ? c0 + c1 : 0.0;
    }
  };
  auto mvt = [&](const double (&u)[R], double (&out)[R]) {
    if constexpr (Gm::REG) {
      out[0] = on[0] ? reg_mv(u[0], Lc) : 0.0;
    } else if constexpr (R == 1 && GL <= 16) {
      double m[K];
      int base = lq + i;
      asm volatile("" : "+v"(base));
#pragma unroll
      for (int k = 0; k < K; ++k) m[k] = smem[base + k * SP];
      out[0] = on[0] ? reg_mv(u[0], m) : 0.0;
    } else if constexpr (GL == 64) {
      // (L^T u)_c for lane c = i: rows r = 16 b + k of column c, b = a ^ s, at r (r + 1) / 2 + c; kept when r >= c
      // (b > a, or b == a and k >= ii) and r < K
      const int a = i >> 4, ii = i & 15;
      double S[4], A, Bv;
      S[0] = u[0];
      pl_swap<16>(u[0], A, Bv);
      S[1] = (a & 1) ? A : Bv;
      pl_swap<32>(u[0], A, Bv);
      S[2] = (a & 2) ? A : Bv;
      pl_swap<32>(S[1], A, Bv);
      S[3] = (a & 2) ? A : Bv;
      double a0 = 0.0, a1 = 0.0;
      if constexpr (Gm::BLK) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int bb = a ^ s;
          const bool lower = bb < Gm::NBK && a <= bb;
          int base = lq + (lower ? bb * (bb + 1) / 2 + a : 0) * 272 + ii;
          asm volatile("" : "+v"(base));
          double m[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) m[k] = smem[base + 17 * k];
          bcf<16, 16>(a0, a1, lower ? S[s] : 0.0, m);
        }
        out[0] = on[0] ? a0 + a1 : 0.0;
        return;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int b = a ^ s;
        int cbase = lq + i + 8 * b * (16 * b + 1);     // column c at row 16 b: T(16 b) + c
        asm volatile("" : "+v"(cbase));
        const bool above = b > a && 16 * b < K;
        double m[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const bool keep = (s == 0 ? k >= ii : above) && 16 * b + k < K;
          m[k] = tri_keep(smem[cbase + 16 * b * k + k * (k + 1) / 2], keep);
        }
        bcf<16, 16>(a0, a1, S[s], m);
      }
      out[0] = on[0] ? a0 + a1 : 0.0;
    } else if constexpr (PK) {
      // columns i and i + 16: L[k][c] at k (k + 1) / 2 + c; above-diagonal entries (k < c) masked
      double m[16], m1[K1], m2[K1];
      int c0i = lq + i, c1i = lq + min(i + 16, K - 1);
      asm volatile("" : "+v"(c0i), "+v"(c1i));
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = tri_keep(smem[c0i + k * (k + 1) / 2], k >= i);
#pragma unroll
      for (int k = 0; k < K1; ++k) {
        m1[k] = smem[c0i + (16 + k) * (17 + k) / 2];
        m2[k] = tri_keep(smem[c1i + (16 + k) * (17 + k) / 2], k >= i);
      }
      double a0 = 0.0, a1 = 0.0, c0 = 0.0, c1 = 0.0;
      bcf<16, 16>(a0, a1, u[0], m);
      bcf<16, K1>(a0, a1, u[1], m1);
      bcf<16, K1>(c0, c1, u[1], m2);
      out[0] = on[0] ? a0 + a1 : 0.0;
      out[1] = on[1] ? c0 + c1 : 0.0;
    } else {
      double m[16], m1[K1], m2[K1];
      int c0i = lq + i, c1i = lq + min(i + 16, K - 1);
      asm volatile("" : "+v"(c0i), "+v"(c1i));
#pragma unroll
      for (int k = 0; k < 16; ++k) m[k] = smem[c0i + k * SP];
#pragma unroll
      for (int k = 0; k < K1; ++k) { m1[k] = smem[c0i + (16 + k) * SP]; m2[k] = smem[c1i + (16 + k) * SP]; }
      double a0 = 0.0, a1 = 0.0, c0 = 0.0, c1 = 0.0;
      bcf<16, 16>(a0, a1, u[0], m);
      bcf<16, K1>(a0, a1, u[1], m1);
      bcf<16, K1>(c0, c1, u[1], m2);
      out[0] = on[0] ? a0 + a1 : 0.0;
      out[1] = on[1] ? c0 + c1 : 0.0;
    }
  };
  auto gsum = [&](const double (&x)[R]) {
    double v = x[0];
    if constexpr (R == 2) v += x[1];
    return group_sum<GL>(v);
  };
  auto vg = [&](const double (&v)[R], double& f, double (&gr)[R], double (&Dw)[R]) {
    double z[R], lt[R], cf[R];
    mv(v, z);
#pragma unroll
    for (int s = 0; s < R; ++s) {
      // response, offset and weight re-read per evaluation (L2 hits; a few evaluations per solve) instead of
      // holding 3 R doubles per lane through the CG loop (VGPRs -> occupancy)
      const double y = on[s] ? Y[o[s]] : 0.0, off = on[s] ? O[o[s]] : 0.0, wt = on[s] ? WT[o[s]] : 0.0;
      double l, dl, d2;
      pointwise_loss(loss, z[s] + off, y, l, dl, d2);
      if (!on[s]) { l = 0.0; dl = 0.0; d2 = 0.0; }
      lt[s] = wt * l + 0.5 * l2 * v[s] * v[s];
      cf[s] = wt * dl;
      Dw[s] = wt * d2;
    }
    f = gsum(lt);
    mvt(cf, gr);
#pragma unroll
    for (int s = 0; s < R; ++s) gr[s] += l2 * v[s];
  };
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75, s1 = 0.25, s2 = 0.5, s3 = 4.0;
  double f, gr[R], Dw[R];
  vg(W, f, gr, Dw);
  double nzw[R];
#pragma unroll
  for (int s = 0; s < R; ++s) nzw[s] = W[s] != 0.0 ? 1.0 : 0.0;
  double f0z, g0n;
  if (gsum(nzw) == 0.0) {
    f0z = f;
    double t[R];
#pragma unroll
    for (int s = 0; s < R; ++s) t[s] = gr[s] * gr[s];
    g0n = sqrt(gsum(t));
  } else {
    double zero[R], f0, g0[R], D0[R], t[R];
#pragma unroll
    for (int s = 0; s < R; ++s) zero[s] = 0.0;
    vg(zero, f0, g0, D0);
    f0z = f0;
#pragma unroll
    for (int s = 0; s < R; ++s) t[s] = g0[s] * g0[s];
    g0n = sqrt(gsum(t));
  }
  const double loss_tol = f0z * tol, grad_tol = g0n * tol;
  double gg[R];
#pragma unroll
  for (int s = 0; s < R; ++s) gg[s] = gr[s] * gr[s];
  double delta = sqrt(gsum(gg));
  int it = 0, fails = 0, reason = 0;
  bool active = prob_on;
  if (delta == 0.0) { reason = 4; active = false; }
  const int guard_max = max_iter * (max_fail + 1) + 5;
  for (int guard = 0; guard < guard_max; ++guard) {
    if (!__any(active)) break;
    // ---- truncated CG at W (Hessian weights Dw of the current iterate)
    double step[R], r[R], d[R], t[R];
#pragma unroll
    for (int s = 0; s < R; ++s) { step[s] = 0.0; r[s] = -gr[s]; d[s] = r[s]; t[s] = r[s] * r[s]; }
    double rtr = gsum(t);
    const double cg_tol = 0.1 * sqrt(rtr);      // ||g|| = ||r0||
    const double cg_tol2 = cg_tol * cg_tol;     // squared tests: no square root per CG step
    double sts = 0.0;                           // ||step||^2
    bool cg_on = active;
    for (int k = 0; k < max_cg; ++k) {
      cg_on = cg_on && rtr > cg_tol2;
      if (!__any(cg_on)) break;
      double u[R], Hl[R];
      mv(d, u);
#pragma unroll
      for (int s = 0; s < R; ++s) u[s] *= Dw[s];
      mvt(u, Hl);
      if constexpr (MS) {
        double sv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < R; ++s) {
          Hl[s] += l2 * d[s];
          sv[0] += d[s] * Hl[s];
          sv[1] += step[s] * d[s];
          sv[2] += d[s] * d[s];
          sv[3] += r[s] * Hl[s];
          sv[4] += Hl[s] * Hl[s];
        }
        group_sum5<GL>(sv);
        const double dhd = sv[0], std_ = sv[1], dtd = sv[2], rh = sv[3], hh = sv[4];
        const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
        double tn = sts + 2.0 * alpha * std_ + alpha * alpha * dtd;
        tn = tn > 0.0 ? tn : 0.0;
        const double dsq = delta * delta;
        const bool hit = tn > dsq;
        double a = alpha;
        if (hit) {
          const double qd = std_ * std_ + dtd * (dsq - sts);
          const double rad = sqrt(qd > 0.0 ? qd : 0.0);
          const double den1 = std_ + rad;
          a = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300)
                          : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
        }
        double rn = rtr - 2.0 * a * rh + a * a * hh;
        rn = rn > 0.0 ? rn : 0.0;
        const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
        if (cg_on) {
#pragma unroll
          for (int s = 0; s < R; ++s) {
            step[s] += a * d[s];
            r[s] -= a * Hl[s];
            if (!hit) d[s] = r[s] + beta * d[s];
          }
          if (!hit) { rtr = rn; sts = tn; }
        }
        cg_on = cg_on && !hit;
        continue;
      }
#pragma unroll
      for (int s = 0; s < R; ++s) { Hl[s] += l2 * d[s]; t[s] = d[s] * Hl[s]; }
      const double dhd = gsum(t);
      const double alpha = rtr / (dhd == 0.0 ? 1.0 : dhd);
      // full step and its residual together (one pair of interleaved sums); a problem that leaves the trust
      // region recomputes its residual at the boundary step (rare: uniform branch)
      double tr[R], rn_[R], t2[R];
#pragma unroll
      for (int s = 0; s < R; ++s) {
        tr[s] = step[s] + alpha * d[s];
        rn_[s] = r[s] - alpha * Hl[s];
        t[s] = tr[s] * tr[s];
        t2[s] = rn_[s] * rn_[s];
      }
      double tn = t[0], rn = t2[0];
      if constexpr (R == 2) { tn += t[1]; rn += t2[1]; }
      group_sum2<GL>(tn, rn);
      const bool hit = tn > delta * delta;
      double a = alpha;
      if (__any(hit && cg_on)) {
#pragma unroll
        for (int s = 0; s < R; ++s) { t[s] = step[s] * d[s]; t2[s] = d[s] * d[s]; }
        double std_ = t[0], dtd = t2[0];
        if constexpr (R == 2) { std_ += t[1]; dtd += t2[1]; }
        group_sum2<GL>(std_, dtd);
        if (hit) {
          const double dsq = delta * delta;
          const double qd = std_ * std_ + dtd * (dsq - sts);
          const double rad = sqrt(qd > 0.0 ? qd : 0.0);
          const double den1 = std_ + rad;
          a = std_ >= 0.0 ? (dsq - sts) / (den1 > 1e-300 ? den1 : 1e-300)
                          : (rad - std_) / (dtd > 1e-300 ? dtd : 1e-300);
        }
#pragma unroll
        for (int s = 0; s < R; ++s) {
          const double rh = r[s] - a * Hl[s];
          rn_[s] = hit ? rh : rn_[s];
          t[s] = rh * rh;
        }
        const double rnh = gsum(t);
        rn = hit ? rnh : rn;
      }
      const double beta = rn / (rtr == 0.0 ? 1.0 : rtr);
      if (cg_on) {
#pragma unroll
        for (int s = 0; s < R; ++s) {
          step[s] = hit ? step[s] + a * d[s] : tr[s];
          r[s] = rn_[s];
          if (!hit) d[s] = rn_[s] + beta * d[s];
        }
        if (!hit) { rtr = rn; sts = tn; }
      }
      cg_on = cg_on && !hit;
    }
    // ---- trial point, trust-region update, acceptance
    double Wn[R], t2[R];
#pragma unroll
    for (int s = 0; s < R; ++s) { Wn[s] = W[s] + step[s]; t[s] = gr[s] * step[s]; t2[s] = step[s] * r[s]; }
    const double gs = gsum(t);
    const double pred = -0.5 * (gs - gsum(t2));
    double fn, gn[R], Dn[R];
    vg(Wn, fn, gn, Dn);
    const double actual = f - fn;
#pragma unroll
    for (int s = 0; s < R; ++s) t[s] = step[s] * step[s];
    const double snorm = sqrt(gsum(t));
    if (active && it == 0) delta = fmin(delta, snorm);
    const double den = fn - f - gs;
    const double al = den <= 0.0 ? s3 : fmax(s1, -0.5 * gs / (den == 0.0 ? 1.0 : den));
    double nd;
    if (actual < eta0 * pred) nd = fmin(fmax(al, s1) * snorm, s2 * delta);
    else if (actual < eta1 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s2 * delta));
    else if (actual < eta2 * pred) nd = fmax(s1 * delta, fmin(al * snorm, s3 * delta));
    else nd = fmax(delta, fmin(al * snorm, s3 * delta));
    if (active) delta = nd;
    const bool accept = active && actual > eta0 * pred;
    const double f_prev = f;
    if (accept) {
#pragma unroll
      for (int s = 0; s < R; ++s) { W[s] = Wn[s]; gr[s] = gn[s]; Dw[s] = Dn[s]; }
      f = fn; ++it; fails = 0;
    } else if (active) {
      ++fails;
    }
    const bool not_impr = active && !accept && fails >= max_fail;
#pragma unroll
    for (int s = 0; s < R; ++s) t[s] = gr[s] * gr[s];
    const double gnorm = sqrt(gsum(t));
    int rc = 0;
    if (accept && gnorm <= grad_tol) rc = 4;
    if (accept && fabs(f - f_prev) <= loss_tol) rc = 3;
    if (not_impr) rc = 2;
    if ((accept || not_impr) && it >= max_iter) rc = 1;
    if (active && rc > 0) { reason = rc; active = false; }
  }
#pragma unroll
  for (int s = 0; s < R; ++s)
    if (on[s]) Beta[o[s]] = W[s];
  if (Zout) {
    // margins of the solution (L beta, no offsets) while L is still resident: the caller's scores need no
    // separate batched GEMV pass that re-reads every L
    double z[R];
    mv(W, z);
#pragma unroll
    for (int s = 0; s < R; ++s)
      if (on[s]) Zout[o[s]] = z[s];
  }
  if (prob_on && i == 0) { Fout[b] = f; Iters[b] = it; Reason[b] = reason; }
}

template <int K, bool LREG, int WL = 2, bool MS = false, bool TRI = false>
static void launch_rs_tron_dpp(int B, int n, const double* L, const double* y, const double* off, const double* wt,
                               double* beta, double* f, int* iters, int* reason, int loss, double l2, double tol,
                               int max_iter, int max_fail, int max_cg, hipStream_t st, const int* order,
                               double* zout) {
  using Gm = RsGeom<K, LREG, WL, TRI>;
  const long long waves = (B + Gm::P - 1) / Gm::P;
  const long long grid = (waves + Gm::WPB - 1) / Gm::WPB;
  const size_t lds = Gm::REG ? 0 : (size_t)Gm::WPB * Gm::P * Gm::PS * sizeof(double);
  hipLaunchKernelGGL((rs_tron_dpp_kernel<K, LREG, WL, MS, TRI>), dim3((unsigned)grid), dim3(Gm::WPB * 64), lds, st, B, n, L, y, off, wt,
                     beta, f, iters, reason, loss, l2, tol, max_iter, max_fail, max_cg, order, zout);
}

// ============================================================================================================
// Margin-space line search (GLM L-BFGS): along x(t) = x0 + t d the margins are affine, z(t) = z0 + t zd with
// z0 = X x0_eff + shift0 + offset (cached by the accepted evaluation) and zd = X d_eff + d_shift (one forward
// pass per iteration). Each trial step then costs one elementwise pass over the rows instead of a full
// forward + transpose pass over the non-zeros:
//   F(t) = sum w l(z(t), y),   D(t) = sum w l'(z(t), y) zd     (phi'(t) = D(t) + l2 x(t).d)
// final = 1 (the accepted t): coef = w l'(z), optional dzz = w l'' and S = sum w l' for the gradient's
// transpose pass; z0 <- z0 + t zd is deferred into the next direction pass (FWD_LS epilogue). Per-block (F, D|S) partials, reduced in a fixed order (deterministic).
// ============================================================================================================
template <typename XT, typename RT>
__global__ __launch_bounds__(NTHREADS) void ls_eval_kernel(int n, double t, int loss, double* __restrict__ z0,
                                                            const double* __restrict__ zd, const RT* __restrict__ y,
                                                            const RT* __restrict__ wt, int final_, XT* __restrict__ coef,
                                                            XT* __restrict__ dzz, double* __restrict__ stats) {
  __shared__ double sh[2 * NTHREADS / 64];
  double F = 0.0, D = 0.0;
  const long long stride = (long long)gridDim.x * NTHREADS;
  // four rows per thread per iteration, all loads issued before the loss arithmetic (memory-level parallelism:
  // one dependent load chain per four rows); the per-thread accumulation order is fixed (deterministic)
  constexpr int LU = 4;
  for (long long i0 = (long long)blockIdx.x * NTHREADS + threadIdx.x; i0 < n; i0 += LU * stride) {
    double zdv[LU], z0v[LU], yv[LU], wv[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const long long i = i0 + u * stride;
      const bool ok = i < n;
      zdv[u] = ok ? zd[i] : 0.0;
      z0v[u] = ok ? z0[i] : 0.0;
      yv[u] = ok ? static_cast<double>(y[i]) : 0.0;
      wv[u] = ok ? static_cast<double>(wt[i]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n) break;
      const double z = z0v[u] + t * zdv[u];
      const double w = wv[u];
      double l, dl, d2;
      pointwise_loss(loss, z, yv[u], l, dl, d2);
      F += wx(w, l);
      if (final_) {
        coef[i] = static_cast<XT>(wx(w, dl));
        if (dzz) dzz[i] = static_cast<XT>(wx(w, d2));
        D += wx(w, dl);
      } else {
        D += wx(w, dl * zdv[u]);
      }
    }
  }
  block_sum2(F, D, sh);
  if (threadIdx.x == 0) { stats[2 * blockIdx.x] = F; stats[2 * blockIdx.x + 1] = D; }
}


// Several trial steps of one line search in ONE pass over the rows: F(t_k), D(t_k) for K step lengths (the strong
// Wolfe search's extrapolation ladder t, 1.5 t, 2.25 t, ... after a first trial that is too short). The rows are
// read once; every (t_k) sum follows exactly the single-step kernel's grid, per-thread row order, block sum and
// reduction, so each (F, D) pair is bitwise what ls_eval_kernel returns for that t alone. stats: [K][2 * nb].
#define LS_MULTI_MAX 6
struct LsTs { double t[LS_MULTI_MAX]; };

template <typename RT, int K>
__global__ __launch_bounds__(NTHREADS) void ls_eval_multi_kernel(int n, LsTs ts, int loss,
                                                                  const double* __restrict__ z0,
                                                                  const double* __restrict__ zd,
                                                                  const RT* __restrict__ y, const RT* __restrict__ wt,
                                                                  double* __restrict__ stats) {
  __shared__ double sh[2 * NTHREADS / 64];
  double F[K], D[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { F[k] = 0.0; D[k] = 0.0; }
  const long long stride = (long long)gridDim.x * NTHREADS;
  constexpr int LU = 4;
  for (long long i0 = (long long)blockIdx.x * NTHREADS + threadIdx.x; i0 < n; i0 += LU * stride) {
    double zdv[LU], z0v[LU], yv[LU], wv[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const long long i = i0 + u * stride;
      const bool ok = i < n;
      zdv[u] = ok ? zd[i] : 0.0;
      z0v[u] = ok ? z0[i] : 0.0;
      yv[u] = ok ? static_cast<double>(y[i]) : 0.0;
      wv[u] = ok ? static_cast<double>(wt[i]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n) break;
      const double w = wv[u];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double t = ts.t[k];
        const double z = z0v[u] + t * zdv[u];
        double l, dl, d2;
        pointwise_loss(loss, z, yv[u], l, dl, d2);
        F[k] += wx(w, l);
        D[k] += wx(w, dl * zdv[u]);
      }
    }
  }
  const int nb = gridDim.x;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double f = F[k], d = D[k];
    block_sum2(f, d, sh);
    if (threadIdx.x == 0) { stats[2 * nb * k + 2 * blockIdx.x] = f; stats[2 * nb * k + 2 * blockIdx.x + 1] = d; }
  }
}

// The strong-Wolfe search's first trial at t = 1 decided ON THE DEVICE, so the gradient pass at the step it would
// accept can be queued right behind the direction pass, gated on this flag (``gate``; the transpose workgroups exit
// at once when it is 0): no host round trip between the two passes. pre = [g.d, d.d, x0.x0, x0.d] (ls_dots), fd =
// (F, D) of the trial (the direction pass's reduction). out = [pre, F, D, accept] for the host, which takes the
// same decision on the same values (line_search.strong_wolfe) and keeps the gated results only when both agree.
// Every expression is the host's, in the host's evaluation order, without contraction.
__global__ void ls_gate_kernel(const double* __restrict__ pre, const double* __restrict__ fd, double f0, double l2,
                               double c1, double c2, double* __restrict__ out, int* __restrict__ gate) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double g0 = pre[0], dd = pre[1], a = pre[2], b = pre[3], t = 1.0;
  double f = fd[0], dphi = fd[1];
  if (l2 > 0.0) {
    f = f + 0.5 * l2 * ((a + 2.0 * t * b) + t * t * dd);
    dphi = dphi + l2 * (b + t * dd);
  }
  int acc = 0;
  if (dd > 0.0 && g0 < 0.0 && isfinite(f) && !(f > f0 + c1 * t * g0) && fabs(dphi) <= -c2 * g0) acc = 1;
  out[0] = g0; out[1] = dd; out[2] = a; out[3] = b; out[4] = fd[0]; out[5] = fd[1]; out[6] = (double)acc;
  *gate = acc;
}

// ------------------------------------------------------------------------------------------------------------
// Gram matrix of a few (k <= 22) long fp64 vectors and their linear combination: the vector-free L-BFGS two-loop
// (optimization/lbfgs.py _History._apply_inverse_gram). The Gram matrix B = V V^T of the k x n basis V is
// GEMM-shaped, so it runs on the fp64 matrix cores (v_mfma_f64_16x16x4f64): the k <= 32 vectors pad to two
// 16-row tiles, and every 4 elements cost three MFMAs per wave (tiles (0,0), (0,1), (1,1); B = A^T, so one
// register per tile serves both operands). Fragments (gfx950): lane l holds V[row = 16 i + (l & 15)][element of
// k-lane l >> 4] for tile i; accumulator q of lane l holds C[(l >> 4) + 4 q][l & 15]. Each wave streams its share of
// the elements straight into registers (64 elements per iteration in 16-B loads, no LDS staging; the LDS-staged
// scalar version was LDS-bound: two LDS reads per FMA, 67 us at n = 1M, k = 21). The 4 waves' tiles are added in
// wave order through LDS and each workgroup writes its partial upper triangle [grid, k (k + 1) / 2] (pair p =
// (a, a + j) in row-major order over a), summed in workgroup order by the consumer: deterministic.
#define GRAM_MAXK 22
#define GRAM_TILE 256            // elements per workgroup tile in the grid formulas (pml_*_grid)
#define GRAM_ES 8                // 16-B loads per vector and lane per wave iteration (2 MFMA k-steps each)
struct VecSet { const double* p[GRAM_MAXK]; double c[GRAM_MAXK]; };
typedef double v4d_g __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gram_kernel(VecSet vs, int k, long long n, double* __restrict__ partial) {
  __shared__ double sm[4][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, sub = lane >> 4;
  // this lane's two vectors (rows r and 16 + r; null past k): uniform loads of the by-value pointer table + selects
  const double* p0 = nullptr;
  const double* p1 = nullptr;
#pragma unroll
  for (int j = 0; j < GRAM_MAXK; ++j) {
    if (j == r && j < k) p0 = vs.p[j];
    if (j == 16 + r && j < k) p1 = vs.p[j];
  }
  v4d_g c00 = {0.0, 0.0, 0.0, 0.0}, c01 = c00, c11 = c00;
  auto step = [&](double x0, double x1) {
    c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x0, c00, 0, 0, 0);
    c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x1, c01, 0, 0, 0);
    c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, x1, c11, 0, 0, 0);
  };
  // Any element order works as long as the element of (k-step, k-lane) does not depend on the row: k-lane ``sub``
  // of load j reads elements e0 + 8 j + 2 sub + {0, 1} (one 16-B load), so the 4 lanes of a row read 64 contiguous
  // bytes per instruction and a wave iteration streams 64 elements of each vector with GRAM_ES 16-B loads in flight.
  constexpr int WE = 8 * GRAM_ES;                       // elements per wave iteration
  const long long stride = (long long)gridDim.x * 4 * WE;
  const long long nfull = n - n % WE;                   // whole wave iterations (16-B aligned pairs)
  typedef double v2d_g __attribute__((ext_vector_type(2)));
  const v2d_g z2 = {0.0, 0.0};
  long long e0 = ((long long)blockIdx.x * 4 + w) * WE;
  for (; e0 < nfull; e0 += stride) {
    v2d_g a0[GRAM_ES], a1[GRAM_ES];
#pragma unroll
    for (int j = 0; j < GRAM_ES; ++j) {
      const long long e = e0 + 8 * j + 2 * sub;
      a0[j] = p0 ? __builtin_nontemporal_load((const v2d_g*)(p0 + e)) : z2;
      a1[j] = p1 ? __builtin_nontemporal_load((const v2d_g*)(p1 + e)) : z2;
    }
#pragma unroll
    for (int j = 0; j < GRAM_ES; ++j) {
      step(a0[j][0], a1[j][0]);
      step(a0[j][1], a1[j][1]);
    }
  }
  if (e0 < n) {                                         // the one partial wave iteration (elements past n are 0)
    for (int j = 0; j < GRAM_ES; ++j)
      for (int h = 0; h < 2; ++h) {
        const long long e = e0 + 8 * j + 2 * sub + h;
        const double x0 = (p0 && e < n) ? p0[e] : 0.0, x1 = (p1 && e < n) ? p1[e] : 0.0;
        step(x0, x1);
      }
  }
  // this wave's 32 x 32 (upper blocks) -> LDS, then the 4 waves added in order
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = sub + 4 * q;
    sm[w][row][r] = c00[q];
    sm[w][row][16 + r] = c01[q];
    sm[w][16 + row][16 + r] = c11[q];
  }
  __syncthreads();
  const int np = k * (k + 1) / 2;
  for (int t = threadIdx.x; t < np; t += 256) {
    int p = t, a = 0;
    while (p >= k - a) { p -= k - a; ++a; }
    const int bb = a + p;
    partial[(long long)blockIdx.x * np + t] = ((sm[0][a][bb] + sm[1][a][bb]) + sm[2][a][bb]) + sm[3][a][bb];
  }
}

__global__ __launch_bounds__(256) void lincomb_kernel(VecSet vs, int k, long long n, double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    double s = 0.0;
    for (int j = 0; j < k; ++j) s = fma(vs.c[j], vs.p[j][i], s);
    out[i] = s;
  }
}

// fixed-order 256-thread block sum: xor butterfly inside each wave, then the 4 wave sums in order (every thread
// gets the result)
__device__ __forceinline__ double tl2_block_sum(double v, double* sh) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();                                   // sh reuse from the previous reduction
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// New L-BFGS history pair in one launch: s = x - x0, y = g - g0 and out = [s.y, y.y, 1/s.y, s.y/y.y, g.g] (g.g: the
// convergence test's gradient norm, fetched in the same host synchronisation). Per-workgroup partial sums; the last
// workgroup to finish (device-scope counter; release/acquire fences make the partials of other XCDs visible) adds
// them in workgroup order (deterministic) and re-arms the counter. Replaces 2 subtractions, 3 dot products
// (6 launches), a stack and 2 scalar divisions.
#define PAIR_GRID 1024
#define PAIR_E 8          // ls_dots: elements per thread per iteration, all loads issued before the first use
typedef double v2d_p __attribute__((ext_vector_type(2)));

// E consecutive elements from i (zeros past n): 16-byte loads when the whole group is in range and p is 16-byte
// aligned (wave-uniform test), else element loads.
template <int E>
__device__ __forceinline__ void load_e(const double* __restrict__ p, long long i, long long n, double (&v)[E]) {
  if (i + E <= n && (((uintptr_t)p) & 15) == 0) {
#pragma unroll
    for (int j = 0; j < E; j += 2) {
      const v2d_p q = *(const v2d_p*)(p + i + j);
      v[j] = q.x;
      v[j + 1] = q.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < E; ++j) v[j] = i + j < n ? p[i + j] : 0.0;
  }
}

__global__ __launch_bounds__(256) void lbfgs_pair_kernel(const double* __restrict__ x, const double* __restrict__ x0,
                                                         const double* __restrict__ g, const double* __restrict__ g0,
                                                         long long n, double* __restrict__ s, double* __restrict__ y,
                                                         double* __restrict__ partial, unsigned* __restrict__ counter,
                                                         double* __restrict__ out) {
  __shared__ double sh[4];
  __shared__ int last;
  double sy = 0.0, yy = 0.0, gg = 0.0;
  // (measured: the 8- and 4-element vector variants of this loop were 12 % and 65 % SLOWER than this one at n = 1M,
  // unlike ls_dots_kernel's, which gained 40 %)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double gi = g[i];
    const double si = x[i] - x0[i], yi = gi - g0[i];
    s[i] = si;
    y[i] = yi;
    sy = fma(si, yi, sy);
    yy = fma(yi, yi, yy);
    gg = fma(gi, gi, gg);
  }
  sy = tl2_block_sum(sy, sh);
  yy = tl2_block_sum(yy, sh);
  gg = tl2_block_sum(gg, sh);
  if (threadIdx.x == 0) {
    partial[3 * blockIdx.x] = sy;
    partial[3 * blockIdx.x + 1] = yy;
    partial[3 * blockIdx.x + 2] = gg;
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double a = 0.0, b = 0.0, c = 0.0;
  for (int j = threadIdx.x; j < (int)gridDim.x; j += 256) {
    a += partial[3 * j];
    b += partial[3 * j + 1];
    c += partial[3 * j + 2];
  }
  a = tl2_block_sum(a, sh);
  b = tl2_block_sum(b, sh);
  c = tl2_block_sum(c, sh);
  if (threadIdx.x == 0) {
    out[0] = a;
    out[1] = b;
    out[2] = 1.0 / a;
    out[3] = a / b;
    out[4] = c;
    *counter = 0u;
  }
}

// The L-BFGS line search's scalars of a new direction d at (x0, g) in one pass: out = [g.d, d.d, x0.x0, x0.d]
// (descent test, first trial 1/||d||, zero-direction test, the L2 terms of the margin line search). Per-workgroup
// partials reduced in workgroup order by the last workgroup (deterministic), as in lbfgs_pair_kernel. Replaces
// four BLAS dot products (eight launches) and a stack.
__global__ __launch_bounds__(256) void ls_dots_kernel(const double* __restrict__ x0, const double* __restrict__ g,
                                                      const double* __restrict__ d, long long n,
                                                      double* __restrict__ partial, unsigned* __restrict__ counter,
                                                      double* __restrict__ out) {
  __shared__ double sh[4];
  __shared__ int last;
  double a = 0.0, b = 0.0, c = 0.0, e = 0.0;
  const long long stride = (long long)gridDim.x * 256 * PAIR_E;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * PAIR_E; i < n; i += stride) {
    double dv[PAIR_E], xv[PAIR_E], gv[PAIR_E];
    load_e(d, i, n, dv);
    load_e(x0, i, n, xv);
    load_e(g, i, n, gv);
#pragma unroll
    for (int j = 0; j < PAIR_E; ++j) {
      a = fma(gv[j], dv[j], a);
      b = fma(dv[j], dv[j], b);
      c = fma(xv[j], xv[j], c);
      e = fma(xv[j], dv[j], e);
    }
  }
  a = tl2_block_sum(a, sh);
  b = tl2_block_sum(b, sh);
  c = tl2_block_sum(c, sh);
  e = tl2_block_sum(e, sh);
  if (threadIdx.x == 0) {
    double* pp = partial + 4 * blockIdx.x;
    pp[0] = a; pp[1] = b; pp[2] = c; pp[3] = e;
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  a = 0.0; b = 0.0; c = 0.0; e = 0.0;
  for (int j = threadIdx.x; j < (int)gridDim.x; j += 256) {
    a += partial[4 * j]; b += partial[4 * j + 1]; c += partial[4 * j + 2]; e += partial[4 * j + 3];
  }
  a = tl2_block_sum(a, sh);
  b = tl2_block_sum(b, sh);
  c = tl2_block_sum(c, sh);
  e = tl2_block_sum(e, sh);
  if (threadIdx.x == 0) {
    out[0] = a; out[1] = b; out[2] = c; out[3] = e;
    *counter = 0u;
  }
}

// L-BFGS two-loop recursion as a chain of 2k + 1 fused step kernels launched back to back from C++ (no host work
// between them; a single cooperative launch with grid barriers was measured slower, profiles/
// lbfgs_device_two_loop_ab.md). Step: x = src (g first, then q); x += sign * c * u; x *= gamma; store x (or -x);
// and the next dot product v . x, reduced by the last workgroup in workgroup order (deterministic) into the next
// coefficient: rho * dot, or a_sub - rho * dot in the second loop. All scalars stay on the device.
struct TwoLoopStep {
  const double* src;      // g (first step) or q
  const double* u;        // update vector (y_j or s_j) or null
  const double* c;        // its coefficient (device scalar) or null
  double sign;            // -1 (first loop) or +1 (second loop)
  const double* gamma;    // scale after the update or null
  const double* v;        // next dot product vector or null
  const double* rho;      // rho of the next coefficient
  const double* a_sub;    // second loop: coefficient = a_sub - rho * dot
  double* out;            // next coefficient
  int negate;             // last step: store -x
};

__global__ __launch_bounds__(256) void lbfgs_step_kernel(TwoLoopStep st, long long n, double* __restrict__ q,
                                                         double* __restrict__ partial, unsigned* __restrict__ counter) {
  __shared__ double sh[4];
  __shared__ int last;
  const double c = st.u ? st.sign * *st.c : 0.0;
  const double gm = st.gamma ? *st.gamma : 1.0;
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    double x = st.src[i];
    if (st.u) x = fma(c, st.u[i], x);
    if (st.gamma) x *= gm;
    q[i] = st.negate ? -x : x;
    if (st.v) acc = fma(st.v[i], x, acc);
  }
  if (!st.v) return;
  acc = tl2_block_sum(acc, sh);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = acc;
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double a = 0.0;
  for (int j = threadIdx.x; j < (int)gridDim.x; j += 256) a += partial[j];
  a = tl2_block_sum(a, sh);
  if (threadIdx.x == 0) {
    const double r = *st.rho * a;
    *st.out = st.a_sub ? *st.a_sub - r : r;
    *counter = 0u;
  }
}


// Vector-free two-loop ON THE DEVICE (Chen, Wang & Zhou 2014): H g is a combination of the basis
// b = [s_0 .. s_{k-1}, y_0 .. y_{k-1}, g]; the recursion runs on the 2k + 1 coefficients using the Gram matrix
// B = b b^T. Three launches and no host synchronisation: gram_kernel (ONE read of the 2k + 1 vectors, per-block
// partials), gram_two_loop_kernel (one workgroup: sums the partials in block order — deterministic — and runs the
// recursion on B in LDS; rho_i = 1 / B[i][k+i], initial scale B[k-1][2k-1] / B[2k-1][2k-1] of the newest pair),
// lincomb_dev_kernel (ONE read of the basis, coefficients from device memory). The step chain it replaces costs
// 2k + 1 dependent launches, each a full pass with a last-workgroup reduction.
#define GTL_THREADS 1024
__global__ __launch_bounds__(GTL_THREADS) void gram_two_loop_kernel(const double* __restrict__ partial, int grid,
                                                                    int k, double* __restrict__ coef, int negate) {
  __shared__ double B[GRAM_MAXK * GRAM_MAXK];
  __shared__ double quarter[4][256];
  const int kk = 2 * k + 1, np = kk * (kk + 1) / 2;
  const int tid = threadIdx.x;
  // pair t = tid & 255 (< np <= 253), quarter qq = tid >> 8 of the workgroup partials: each thread sums its quarter
  // of the rows with 8 interleaved accumulators (independent loads in flight; a single thread per pair over all
  // rows was a 30 us latency chain), then the quarters are added in order (deterministic)
  const int t = tid & 255, qq = tid >> 8;
  if (t < np) {
    const int g0 = (grid * qq) / 4, g1 = (grid * (qq + 1)) / 4;
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int g = g0;
    for (; g + 8 <= g1; g += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += partial[(long long)(g + u) * np + t];
    }
    for (int u = 0; g + u < g1; ++u) acc[u] += partial[(long long)(g + u) * np + t];
    quarter[qq][t] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  __syncthreads();
  if (tid < np) {
    const double s = ((quarter[0][tid] + quarter[1][tid]) + quarter[2][tid]) + quarter[3][tid];
    int p = tid, a = 0;
    while (p >= kk - a) { p -= kk - a; ++a; }
    B[a * kk + a + p] = s;
    B[(a + p) * kk + a] = s;
  }
  __syncthreads();
  if (tid >= 64) return;
  // the recursion on wave 0: lane j holds delta[j]; each dot product is one fixed-order wave sum (no per-thread
  // arrays indexed at run time, which went to scratch memory)
  const int j = tid;
  const bool on = j < kk;
  double delta = (j == 2 * k) ? 1.0 : 0.0;
  double alpha_mine = 0.0;                    // lane i keeps alpha_i
  for (int i = k - 1; i >= 0; --i) {
    const double dot = wave_sum(on ? delta * B[j * kk + i] : 0.0);          // s_i . q
    const double al = dot / B[i * kk + k + i];                               // rho_i = 1 / (s_i . y_i)
    if (j == i) alpha_mine = al;
    if (j == k + i) delta -= al;
  }
  delta *= B[(k - 1) * kk + 2 * k - 1] / B[(2 * k - 1) * kk + 2 * k - 1];
  for (int i = 0; i < k; ++i) {
    const double dot = wave_sum(on ? delta * B[j * kk + k + i] : 0.0);      // y_i . r
    if (j == i) delta += alpha_mine - dot / B[i * kk + k + i];
  }
  if (on) coef[j] = negate ? -delta : delta;
}

__global__ __launch_bounds__(256) void lincomb_dev_kernel(VecSet vs, int k, long long n, const double* __restrict__ coef,
                                                          double* __restrict__ out) {
  double c[GRAM_MAXK];
#pragma unroll
  for (int j = 0; j < GRAM_MAXK; ++j) c[j] = j < k ? coef[j] : 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < GRAM_MAXK; ++j)
      if (j < k) s = fma(c[j], vs.p[j][i], s);
    out[i] = s;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Per-iteration vector epilogues of the GLM line search (one launch each instead of a torch op chain):
// * perm_cast_kernel: the coefficient vector in the shard's device column order and gather precision,
//   out[i] = (XT) w[perm[i]] (perm null: a cast) — the input of every forward pass (was an index gather + a cast);
// * ls_step_grad_kernel: the accepted step x = x0 + t d and the full gradient g = G[perm[i]] + l2 x (perm null:
//   G[i]), with G the transpose pass's result in device column order (was an index_select, two scaled adds and
//   two more elementwise kernels). Products and sums are rounded separately (no FMA contraction), so x and g are
//   bitwise the values of the torch expressions x0 + t * d and g + l2 * x they replace.
template <typename XT>
__global__ __launch_bounds__(256) void perm_cast_kernel(const double* __restrict__ w, const long long* __restrict__ perm,
                                                         long long n, XT* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    out[i] = static_cast<XT>(perm ? w[perm[i]] : w[i]);
}

// out[i] = src[idx[i]] (0 where idx[i] < 0): packed per-slot values of a per-row vector (row-space batches:
// padding slots carry index -1) in one pass instead of a clamp, a gather and a select.
__global__ __launch_bounds__(256) void masked_gather_kernel(const double* __restrict__ src,
                                                            const long long* __restrict__ idx, long long n,
                                                            double* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long j = idx[i];
    out[i] = j >= 0 ? src[j] : 0.0;
  }
}

// GAME fixed-effect offsets for the next update in one pass: o = (RT)(base + partial) and, when the cached margins
// are kept, z += (double) o_new - (double) o_old (the margins shift by the offset change) -- the torch chain it
// replaces (an add, a cast, two casts, a subtraction, an in-place add, a copy) rounded the same way.
template <typename RT>
__global__ __launch_bounds__(256) void offset_update_kernel(const double* __restrict__ base,
                                                            const double* __restrict__ part, long long n,
                                                            RT* __restrict__ o, double* __restrict__ z) {
#pragma clang fp contract(off)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const RT nw = static_cast<RT>(base[i] + part[i]);
    if (z) z[i] = z[i] + (static_cast<double>(nw) - static_cast<double>(o[i]));
    o[i] = nw;
  }
}

// Scores of the optimizer's last accepted point from the cached margins: out = (z0 + t zd) [- o] in one pass
// (DeviceGLMData.margins; the torch sequence clone / add_(alpha = t) / cast / sub_ was four passes). z0 + t zd is
// one fma (one rounding), then the offset subtraction.
template <typename RT>
__global__ __launch_bounds__(256) void cached_margins_kernel(const double* __restrict__ z0,
                                                             const double* __restrict__ zd, double t,
                                                             const RT* __restrict__ o, long long n,
                                                             double* __restrict__ out) {
#pragma clang fp contract(off)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    double z = z0[i];
    if (zd) z = fma(t, zd[i], z);
    if (o) z = z - static_cast<double>(o[i]);
    out[i] = z;
  }
}

__global__ __launch_bounds__(256) void ls_step_grad_kernel(const double* __restrict__ x0, const double* __restrict__ d,
                                                           double t, const double* __restrict__ G,
                                                           const long long* __restrict__ perm, double l2, long long n,
                                                           double* __restrict__ x, double* __restrict__ g) {
#pragma clang fp contract(off)   // (HIP's __dmul_rn / __dadd_rn are plain operators: no FMA contraction here)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double xi = x0[i] + t * d[i];
    x[i] = xi;
    const double gi = perm ? G[perm[i]] : G[i];
    g[i] = l2 != 0.0 ? gi + l2 * xi : gi;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Determinism probe for the one ISA-unpinned assumption above: the order in which the LDS applies the lanes of ONE
// ds_add_f64 instruction that all hit the same address. Trial t: the 64 lanes of a wave add v[t][lane] (values of
// widely spread magnitudes, so the rounded sum depends on the order) into one LDS double. The host compares the
// results with the lane-ascending sequential sum (ops.native.check_lds_add_order), once per process.
__global__ __launch_bounds__(64) void lds_add_order_probe_kernel(const double* __restrict__ v, double* __restrict__ out,
                                                                 int trials) {
  __shared__ double cell;
  for (int t = 0; t < trials; ++t) {
    if (threadIdx.x == 0) cell = 0.0;
    __syncthreads();
    atomicAdd(&cell, v[t * 64 + threadIdx.x]);
    __syncthreads();
    if (threadIdx.x == 0) out[t] = cell;
    __syncthreads();
  }
}

extern "C" {

const char* pml_build_id() { return pml_build_stamp + 13; }

// H g (negate: -H g) for a k-deep history (newest last): rho[j] = 1/s_j.y_j and gamma = s.y/y.y of the newest
// pair are device scalars; coef: 2k doubles of device scratch; partial: 1024 doubles; counter: one zeroed unsigned.
int pml_two_loop_chain(int k, const double* const* s, const double* const* y, const double* const* rho,
                       const double* gamma, const double* g, long long n, double* q, double* coef, double* partial,
                       unsigned* counter, int negate, void* stream) {
  if (k < 1 || n <= 0) return -22;
  const int grid = (int)std::min<long long>(PAIR_GRID, (n + 255) / 256);
  double* alpha = coef;           // alpha[j]
  double* cc = coef + k;          // alpha[j] - beta[j]
  auto launch = [&](const TwoLoopStep& st) {
    hipLaunchKernelGGL(lbfgs_step_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, st, n, q, partial, counter);
  };
  // q = g; alpha[k-1] = rho (s_{k-1} . q)
  launch(TwoLoopStep{g, nullptr, nullptr, 0.0, nullptr, s[k - 1], rho[k - 1], nullptr, alpha + k - 1, 0});
  for (int j = k - 1; j >= 1; --j)   // q -= alpha_j y_j; alpha[j-1] = rho (s_{j-1} . q)
    launch(TwoLoopStep{q, y[j], alpha + j, -1.0, nullptr, s[j - 1], rho[j - 1], nullptr, alpha + j - 1, 0});
  // q -= alpha_0 y_0; q *= gamma; c[0] = alpha_0 - rho_0 (y_0 . q)
  launch(TwoLoopStep{q, y[0], alpha, -1.0, gamma, y[0], rho[0], alpha, cc, 0});
  for (int j = 0; j + 1 < k; ++j)    // q += c_j s_j; c[j+1] = alpha_{j+1} - rho_{j+1} (y_{j+1} . q)
    launch(TwoLoopStep{q, s[j], cc + j, 1.0, nullptr, y[j + 1], rho[j + 1], alpha + j + 1, cc + j + 1, 0});
  launch(TwoLoopStep{q, s[k - 1], cc + k - 1, 1.0, nullptr, nullptr, nullptr, nullptr, nullptr, negate});
  LAUNCH_CHECK();
  return 0;
}

// Grid of the device vector-free two-loop's Gram pass (partial buffer: grid x (2k+1)(2k+2)/2 doubles).
int pml_two_loop_gram_grid(long long n) {
  const long long t = (n + GRAM_TILE - 1) / GRAM_TILE;
  return (int)std::max<long long>(1, std::min<long long>(t, 512));
}

int pml_two_loop_gram(int k, const double* const* s, const double* const* y, const double* g, long long n, double* q,
                      double* partial, double* coef, int negate, void* stream) {
  if (k < 1 || 2 * k + 1 > GRAM_MAXK || n <= 0) return -22;
  VecSet vs{};
  for (int j = 0; j < k; ++j) { vs.p[j] = s[j]; vs.p[k + j] = y[j]; }
  vs.p[2 * k] = g;
  const int kk = 2 * k + 1, grid = pml_two_loop_gram_grid(n);
  hipLaunchKernelGGL(gram_kernel, dim3(grid), dim3(GRAM_TILE), 0, (hipStream_t)stream, vs, kk, n, partial);
  hipLaunchKernelGGL(gram_two_loop_kernel, dim3(1), dim3(GTL_THREADS), 0, (hipStream_t)stream, partial, grid, k, coef,
                     negate);
  const long long blocks = std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(lincomb_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, vs, kk, n, coef, q);
  LAUNCH_CHECK();
  return 0;
}

// out[4] = [g.d, d.d, x0.x0, x0.d]; partial: 4 * 1024 doubles; counter: one zeroed unsigned (re-armed).
int pml_ls_dots(const double* x0, const double* g, const double* d, long long n, double* partial, unsigned* counter,
                double* out, void* stream) {
  if (n <= 0) return -22;
  const int grid = (int)std::min<long long>(PAIR_GRID, (n + 256 * PAIR_E - 1) / (256 * PAIR_E));
  hipLaunchKernelGGL(ls_dots_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x0, g, d, n, partial, counter,
                     out);
  LAUNCH_CHECK();
  return 0;
}

// s = x - x0, y = g - g0, out[5] = [s.y, y.y, 1/s.y, s.y/y.y, g.g]; partial: 3 * 1024 doubles; counter: one zeroed
// unsigned (re-armed by the kernel).
int pml_lbfgs_pair(const double* x, const double* x0, const double* g, const double* g0, long long n, double* s,
                   double* y, double* partial, unsigned* counter, double* out, void* stream) {
  if (n <= 0) return -22;
  const int grid = (int)std::min<long long>(PAIR_GRID, (n + 255) / 256);
  hipLaunchKernelGGL(lbfgs_pair_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, x0, g, g0, n, s, y, partial,
                     counter, out);
  LAUNCH_CHECK();
  return 0;
}

static int vec_grid(long long n) { return (int)std::min<long long>(8192, (n + 255) / 256); }

// prec: 2 -> fp64 output, else fp32 (the forward pass's gather precision)
int pml_perm_cast(const double* w, const long long* perm, long long n, int prec, void* out, void* stream) {
  if (n <= 0) return 0;
  if (prec == 2)
    hipLaunchKernelGGL(perm_cast_kernel<double>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, w, perm, n,
                       (double*)out);
  else
    hipLaunchKernelGGL(perm_cast_kernel<float>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, w, perm, n,
                       (float*)out);
  LAUNCH_CHECK();
  return 0;
}

int pml_masked_gather(const double* src, const long long* idx, long long n, double* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(masked_gather_kernel, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, src, idx, n, out);
  LAUNCH_CHECK();
  return 0;
}

// prec 2: fp64 row vectors, else fp32; z may be null (no margin cache)
int pml_offset_update(const double* base, const double* part, long long n, int prec, void* o, double* z,
                      void* stream) {
  if (n <= 0) return 0;
  if (prec == 2)
    hipLaunchKernelGGL(offset_update_kernel<double>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, base, part,
                       n, (double*)o, z);
  else
    hipLaunchKernelGGL(offset_update_kernel<float>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, base, part,
                       n, (float*)o, z);
  LAUNCH_CHECK();
  return 0;
}

int pml_cached_margins(const double* z0, const double* zd, double t, int prec, const void* o, long long n,
                       double* out, void* stream) {
  if (n <= 0) return 0;
  if (prec == 2 || o == nullptr)
    hipLaunchKernelGGL(cached_margins_kernel<double>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, z0, zd,
                       t, (const double*)o, n, out);
  else
    hipLaunchKernelGGL(cached_margins_kernel<float>, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, z0, zd,
                       t, (const float*)o, n, out);
  LAUNCH_CHECK();
  return 0;
}

int pml_ls_step_grad(const double* x0, const double* d, double t, const double* G, const long long* perm, double l2,
                     long long n, double* x, double* g, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ls_step_grad_kernel, dim3(vec_grid(n)), dim3(256), 0, (hipStream_t)stream, x0, d, t, G, perm,
                     l2, n, x, g);
  LAUNCH_CHECK();
  return 0;
}

int pml_version() { return 1; }
void pml_tl_set_deep(int fwd, int t) { g_tl_deep = fwd; g_tl_deep_t = t; }

void pml_set_ls_args(double* z0, double t0, double tpend) { g_ls_z0 = z0; g_ls_t0 = t0; g_ls_tpend = tpend; }
void pml_set_ls_in(const double* z0_in, const double* zd_in) { g_ls_z0_in = z0_in; g_ls_zd_in = zd_in; }
void pml_set_gate(const int* gate) { g_gate = gate; }
int pml_ls_gate(const double* pre, const double* fd, double f0, double l2, double c1, double c2, double* out,
                int* gate, void* stream) {
  hipLaunchKernelGGL(ls_gate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, pre, fd, f0, l2, c1, c2, out, gate);
  LAUNCH_CHECK();
  return 0;
}

void pml_set_ablate(int a) {
  g_ablate = a;
#ifdef PML_TL_EXPERIMENT
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_tl_ablate), &a, sizeof(int));
#endif
}
// layout: 0 = vector, 1 = strided; grid: persistent forward grid size (workgroups)
void pml_set_config(int fwd_strided, int t_strided, int hot_n, int fwd_grid) {
  g_fwd_strided = fwd_strided; g_t_strided = t_strided; g_hot_n = hot_n;
  if (fwd_grid > 0) g_fwd_grid = fwd_grid;
}
int pml_nb() { return NB; }
int pml_maxseg() { return MAXSEG; }
int pml_maxseg_fwd() { return MAXSEG_FWD; }

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
                              (double*)coef, (double*)dzz, z_out, with_offset, g_ablate, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
    return fwd_impl<double, double, double, double>(c, x, with_ls_in(a), stats, long_stats, parts, st);
  }
  FwdArgs<float, float> a{mode, loss, shift, (const float*)y, (const float*)off, (const float*)wt,
                          (float*)coef, (float*)dzz, z_out, with_offset, g_ablate, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
  if (prec == 1) return fwd_impl<float, float, float, float>(c, x, with_ls_in(a), stats, long_stats, parts, st);
  return fwd_impl<uint16_t, float, float, float>(c, x, with_ls_in(a), stats, long_stats, parts, st);
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

// ---- tiled layout entry points ------------------------------------------------------------------------------
int pml_tl_maxbits() { return TL_MAXBITS; }
int pml_tl_experiment() { return TL_KNOB(1); }
void pml_tl_config(int acc64, int waves, int waves_t, int pipe) {
  g_tl_acc64 = acc64; g_tl_waves = (waves == 1 || waves == 2) ? waves : 4; g_tl_waves_t = waves_t == 2 ? 2 : 4; g_tl_pipe = pipe & 3; g_tl_pipe_t = (pipe >> 2) & 3;
}

int pml_tl_fwd(int prec, const TLFwdDesc* c, const void* x, int mode, int loss, double shift, const void* y,
               const void* off, const void* wt, void* coef, void* dzz, double* z_out, int with_offset,
               double* stats, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) {
    FwdArgs<double, double> a{mode, loss, shift, (const double*)y, (const double*)off, (const double*)wt,
                              (double*)coef, (double*)dzz, z_out, with_offset, g_ablate, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
    return tl_fwd_impl<double, double, double>(c, x, with_ls_in(a), stats, st);
  }
  FwdArgs<float, float> a{mode, loss, shift, (const float*)y, (const float*)off, (const float*)wt,
                          (float*)coef, (float*)dzz, z_out, with_offset, g_ablate, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
  if (prec == 1) return tl_fwd_impl<float, float, float>(c, x, with_ls_in(a), stats, st);
  return tl_fwd_impl<uint16_t, float, float>(c, x, with_ls_in(a), stats, st);
}

int pml_tl_t(int prec, const TLTDesc* c, const void* x, int square, double* G, double* parts, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) return square ? tl_t_impl<double, double, true>(c, x, G, parts, st)
                               : tl_t_impl<double, double, false>(c, x, G, parts, st);
  if (prec == 1) return square ? tl_t_impl<float, float, true>(c, x, G, parts, st)
                               : tl_t_impl<float, float, false>(c, x, G, parts, st);
  return square ? tl_t_impl<uint16_t, float, true>(c, x, G, parts, st)
                : tl_t_impl<uint16_t, float, false>(c, x, G, parts, st);
}

int pml_tl_t_multi(int prec, const TLTMultiDesc* c, const void* x, int square, double* G, double* parts,
                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) return square ? tl_t_multi_impl<double, double, true>(c, x, G, parts, st)
                               : tl_t_multi_impl<double, double, false>(c, x, G, parts, st);
  if (prec == 1) return square ? tl_t_multi_impl<float, float, true>(c, x, G, parts, st)
                               : tl_t_multi_impl<float, float, false>(c, x, G, parts, st);
  return square ? tl_t_multi_impl<uint16_t, float, true>(c, x, G, parts, st)
                : tl_t_multi_impl<uint16_t, float, false>(c, x, G, parts, st);
}

int pml_seg_cg_step(const long long* ptr, int nseg, double* step, double* r, double* d, const double* Hd,
                    double* rtr, unsigned char* on, const double* delta, double l2, void* stream) {
  if (nseg <= 0) return 0;
  const int per = NTHREADS / 64;
  hipLaunchKernelGGL(seg_cg_step_kernel, dim3((nseg + per - 1) / per), dim3(NTHREADS), 0, (hipStream_t)stream, ptr,
                     nseg, step, r, d, Hd, rtr, on, delta, l2);
  LAUNCH_CHECK();
  return 0;
}

int pml_seg_expand(const long long* ptr, int nseg, const void* src, void* out, int elem_bytes, void* stream) {
  if (nseg <= 0) return 0;
  const int per = NTHREADS / 64;
  const dim3 grid((nseg + per - 1) / per);
  if (elem_bytes == 8)
    hipLaunchKernelGGL(seg_expand_kernel<unsigned long long>, grid, dim3(NTHREADS), 0, (hipStream_t)stream, ptr, nseg,
                       (const unsigned long long*)src, (unsigned long long*)out);
  else if (elem_bytes == 1)
    hipLaunchKernelGGL(seg_expand_kernel<unsigned char>, grid, dim3(NTHREADS), 0, (hipStream_t)stream, ptr, nseg,
                       (const unsigned char*)src, (unsigned char*)out);
  else
    return -22;
  LAUNCH_CHECK();
  return 0;
}

// Gram: partial [grid, k(k+1)/2] (grid = pml_gram_grid(n)); the caller sums over the grid.
int pml_gram_grid(long long n) {
  const long long t = (n + GRAM_TILE - 1) / GRAM_TILE;
  return (int)std::max<long long>(1, std::min<long long>(t, 2048));
}

int pml_gram(const double* const* ptrs, int k, long long n, double* partial, void* stream) {
  if (k < 1 || k > GRAM_MAXK || n < 0) return -22;
  VecSet vs{};
  for (int j = 0; j < k; ++j) vs.p[j] = ptrs[j];
  hipLaunchKernelGGL(gram_kernel, dim3(pml_gram_grid(n)), dim3(GRAM_TILE), 0, (hipStream_t)stream, vs, k, n,
                     partial);
  LAUNCH_CHECK();
  return 0;
}

int pml_lincomb(const double* const* ptrs, const double* coefs, int k, long long n, double* out, void* stream) {
  if (k < 1 || k > GRAM_MAXK || n < 0) return -22;
  if (n == 0) return 0;
  VecSet vs{};
  for (int j = 0; j < k; ++j) { vs.p[j] = ptrs[j]; vs.c[j] = coefs[j]; }
  const long long blocks = std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, vs, k, n, out);
  LAUNCH_CHECK();
  return 0;
}

int pml_btrsv(int B, int n, const double* L, const double* x, double* y, int trans, void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 192) return -22;
  int G = 1;
  while (G < n && G < 64) G <<= 1;
  const int P = 64 / G;
  hipLaunchKernelGGL(btrsv_kernel, dim3((unsigned)((B + P - 1) / P)), dim3(64),
                     (size_t)P * (n * (n + 1) / 2 + n) * sizeof(double), (hipStream_t)stream, B, n, G, L, x, y, trans);
  LAUNCH_CHECK();
  return 0;
}

int pml_bgemv(int B, int n, const double* A, const double* x, double* y, int trans, void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 192) return -22;
  if (n > 64) {
    hipLaunchKernelGGL(bgemv_wide_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, B, n, A,
                       x, y, trans);
    LAUNCH_CHECK();
    return 0;
  }
  const long long waves = (B + (64 / n) - 1) / (64 / n);
  const size_t wave_lds = (size_t)(64 / n) * n * (n + 1) * sizeof(double);
  const int nw = (int)std::max<size_t>(1, std::min<size_t>(4, 65536 / wave_lds));  // <= 64 KB LDS per workgroup
  const long long grid = (waves + nw - 1) / nw;
  const size_t lds = nw * wave_lds;
  hipLaunchKernelGGL(bgemv_kernel, dim3((unsigned)grid), dim3(nw * 64), lds, (hipStream_t)stream, B, n, A, x, y,
                     trans);
  LAUNCH_CHECK();
  return 0;
}

int pml_bhv(int B, int n, const double* A, const double* dw, const double* v, double l2, double* out, void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 64) return -22;
  const long long waves = (B + (64 / n) - 1) / (64 / n);
  const size_t wave_lds = (size_t)(64 / n) * n * (n + 1) * sizeof(double);
  const int nw = (int)std::max<size_t>(1, std::min<size_t>(4, 65536 / wave_lds));  // <= 64 KB LDS per workgroup
  const long long grid = (waves + nw - 1) / nw;
  const size_t lds = nw * wave_lds;
  hipLaunchKernelGGL(bhv_kernel, dim3((unsigned)grid), dim3(nw * 64), lds, (hipStream_t)stream, B, n, A, dw, v, l2,
                     out);
  LAUNCH_CHECK();
  return 0;
}

void pml_rs_set_variant(int v) { g_rs_variant = v; }

// order (optional, n <= 32 kernels): a permutation of the B problems; waves take consecutive problems of it
// (a scheduling hint only: results land in each problem's own slot whatever the order)
int pml_rs_tron(int B, int n, const double* L, const double* y, const double* off, const double* wt, double* beta,
                double* f, int* iters, int* reason, int loss, double l2, double tol, int max_iter, int max_fail,
                int max_cg, const int* order, double* zout, void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 64 || loss < 0 || loss > 2) return -22;
  const int V = g_rs_variant;
  hipStream_t st = (hipStream_t)stream;
  if (V >= 3 && n <= 32) {
#define RS_DPP(KK)                                                                                              \
  (V == 3 ? launch_rs_tron_dpp<KK, true>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol, max_iter,    \
                                         max_fail, max_cg, st, order, zout)                                              \
   : (V == 5 || V == 8) ? (KK > 20 ? launch_rs_tron_dpp<KK, true, 1, false, true>(B, n, L, y, off, wt, beta, f, iters, reason,  \
                                                                     loss, l2, tol, max_iter, max_fail, max_cg, st,    \
                                                                     order, zout)                                      \
                        : launch_rs_tron_dpp<KK, true, 1>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol,  \
                                                          max_iter, max_fail, max_cg, st, order, zout))                \
   : V == 6 ? launch_rs_tron_dpp<KK, true, 1, true>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol,    \
                                                    max_iter, max_fail, max_cg, st, order, zout)                         \
   : V == 7 ? launch_rs_tron_dpp<KK, true, 1, false, true>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, \
                                                           tol, max_iter, max_fail, max_cg, st, order, zout)             \
          : launch_rs_tron_dpp<KK, false>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol, max_iter,   \
                                          max_fail, max_cg, st, order, zout))
    if (n <= 4) RS_DPP(4);
    else if (n <= 8) RS_DPP(8);
    else if (n <= 12) RS_DPP(12);
    else if (n <= 16) RS_DPP(16);
    else if (n <= 20) RS_DPP(20);
    else if (n <= 24) RS_DPP(24);
    else RS_DPP(32);
#undef RS_DPP
    LAUNCH_CHECK();
    return 0;
  }
  // n in (32, 64]: one problem per wave, DPP-broadcast FMAs over permlane-rotated column blocks (variant 8, the
  // default: 1.57x at n = 64, 1.15x at n = 48 over rs_tron_kernel<2>; profiles/rs_tron_roofline.md)
  if ((V == 5 || V == 8) && n > 32) {
    if (n <= 48)
      launch_rs_tron_dpp<48, false, 1, false, true>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol,
                                                    max_iter, max_fail, max_cg, st, order, zout);
    else
      launch_rs_tron_dpp<64, false, 1, false, true>(B, n, L, y, off, wt, beta, f, iters, reason, loss, l2, tol,
                                                    max_iter, max_fail, max_cg, st, order, zout);
    LAUNCH_CHECK();
    return 0;
  }
  int G = 1;
  while (G < n) G <<= 1;
  const int per = 64 / G;
  const long long waves = (B + per - 1) / per;
  const size_t wave_lds = (size_t)per * (n * (n + 1) / 2 + (V >= 1 ? G : 0)) * sizeof(double);
  const int nw = (int)std::max<size_t>(1, std::min<size_t>(4, 65536 / wave_lds));
  const long long grid = (waves + nw - 1) / nw;
  if (V >= 2)
    hipLaunchKernelGGL(rs_tron_kernel<2>, dim3((unsigned)grid), dim3(nw * 64), nw * wave_lds, (hipStream_t)stream, B,
                       n, G, L, y, off, wt, beta, f, iters, reason, loss, l2, tol, max_iter, max_fail, max_cg, zout);
  else if (V == 1)
    hipLaunchKernelGGL(rs_tron_kernel<1>, dim3((unsigned)grid), dim3(nw * 64), nw * wave_lds, (hipStream_t)stream, B,
                       n, G, L, y, off, wt, beta, f, iters, reason, loss, l2, tol, max_iter, max_fail, max_cg, zout);
  else
    hipLaunchKernelGGL(rs_tron_kernel<0>, dim3((unsigned)grid), dim3(nw * 64), nw * wave_lds, (hipStream_t)stream, B,
                       n, G, L, y, off, wt, beta, f, iters, reason, loss, l2, tol, max_iter, max_fail, max_cg, zout);
  LAUNCH_CHECK();
  return 0;
}

// Margin-space line-search evaluation; out[0..1] = (F, D) or (F, S) when final. stats: >= 2 * 4096 doubles.
int pml_ls_eval(int prec, int n, double t, int loss, double* z0, const double* zd, const void* y, const void* wt,
                int final_, void* coef, void* dzz, double* stats, double* out, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // up to 4096 workgroups (16 per CU): the per-row loss is a dependent fp64 exp / log1p / reciprocal chain, more
  // waves in flight hide it (stats: >= 2 * 4096 doubles)
  const int nb = (int)std::min<long long>(4096, ((long long)n + 4 * NTHREADS - 1) / (4 * NTHREADS));
  if (prec == 2)
    hipLaunchKernelGGL((ls_eval_kernel<double, double>), dim3(nb), dim3(NTHREADS), 0, st, n, t, loss, z0, zd,
                       (const double*)y, (const double*)wt, final_, (double*)coef, (double*)dzz, stats);
  else
    hipLaunchKernelGGL((ls_eval_kernel<float, float>), dim3(nb), dim3(NTHREADS), 0, st, n, t, loss, z0, zd,
                       (const float*)y, (const float*)wt, final_, (float*)coef, (float*)dzz, stats);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(NTHREADS), 0, st, stats, nb, out, 0);
  LAUNCH_CHECK();
  return 0;
}

// ls_eval at K <= LS_MULTI_MAX step lengths in one pass: out[2k .. 2k + 1] = (F, D) at ts[k], each bitwise the
// single-step result. stats: >= K * 2 * 4096 doubles.
int pml_ls_eval_multi(int prec, int n, int K, const double* ts, int loss, const double* z0, const double* zd,
                      const void* y, const void* wt, double* stats, double* out, void* stream) {
  if (n <= 0) return 0;
  if (K < 1 || K > LS_MULTI_MAX) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)std::min<long long>(4096, ((long long)n + 4 * NTHREADS - 1) / (4 * NTHREADS));   // as pml_ls_eval
  LsTs a;
  for (int k = 0; k < LS_MULTI_MAX; ++k) a.t[k] = k < K ? ts[k] : 0.0;
#define LSM(RT_, K_) hipLaunchKernelGGL((ls_eval_multi_kernel<RT_, K_>), dim3(nb), dim3(NTHREADS), 0, st, n, a, loss, \
                                        z0, zd, (const RT_*)y, (const RT_*)wt, stats)
#define LSM_K(RT_) switch (K) { case 1: LSM(RT_, 1); break; case 2: LSM(RT_, 2); break; case 3: LSM(RT_, 3); break; \
                                case 4: LSM(RT_, 4); break; case 5: LSM(RT_, 5); break; default: LSM(RT_, 6); break; }
  if (prec == 2) { LSM_K(double) } else { LSM_K(float) }
#undef LSM_K
#undef LSM
  LAUNCH_CHECK();
  for (int k = 0; k < K; ++k) {
    hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(NTHREADS), 0, st, stats + 2 * nb * k, nb, out + 2 * k, 0);
    LAUNCH_CHECK();
  }
  return 0;
}

int pml_segdot(const double* a, const double* b, int mode, const long long* ptr, int nseg, double* out,
               void* stream) {
  if (nseg <= 0) return 0;
  const int per = NTHREADS / 64;
  hipLaunchKernelGGL(segdot_kernel, dim3((nseg + per - 1) / per), dim3(NTHREADS), 0, (hipStream_t)stream, a, b,
                     mode, ptr, nseg, out);
  LAUNCH_CHECK();
  return 0;
}

// segments longer than SEGDOT_C present (the caller knows its segment table): scratch >= 2 ceil(n / SEGDOT_C)
int pml_segdot_long(const double* a, const double* b, int mode, const long long* ptr, int nseg, long long n,
                    double* scratch, double* out, void* stream) {
  if (nseg <= 0) return 0;
  const int per = NTHREADS / 64;
  const long long nch = (n + SEGDOT_C - 1) / SEGDOT_C;
  const long long nseg_w = ((long long)nseg + per - 1) / per * per;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(segdot_long_kernel, dim3((unsigned)((nseg_w + nch + per - 1) / per)), dim3(NTHREADS), 0, st, a, b,
                     mode, ptr, nseg, (int)nseg_w, n, scratch, scratch + nch, out);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(segdot_combine_kernel, dim3((nseg + NTHREADS - 1) / NTHREADS), dim3(NTHREADS), 0, st, ptr, nseg,
                     scratch, scratch + nch, out);
  LAUNCH_CHECK();
  return 0;
}

int pml_tl_fwd_multi(int prec, const TLFwdMultiDesc* c, const void* x, int mode, int loss, double shift,
                     const void* y, const void* off, const void* wt, void* coef, void* dzz, double* z_out,
                     int with_offset, double* stats, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (prec == 2) {
    FwdArgs<double, double> a{mode, loss, shift, (const double*)y, (const double*)off, (const double*)wt,
                              (double*)coef, (double*)dzz, z_out, with_offset, 0, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
    return tl_fwd_multi_impl<double, double, double>(c, x, with_ls_in(a), stats, st);
  }
  FwdArgs<float, float> a{mode, loss, shift, (const float*)y, (const float*)off, (const float*)wt,
                          (float*)coef, (float*)dzz, z_out, with_offset, 0, 0, g_ls_z0, g_ls_t0, g_ls_tpend};
  if (prec == 1) return tl_fwd_multi_impl<float, float, float>(c, x, with_ls_in(a), stats, st);
  return tl_fwd_multi_impl<uint16_t, float, float>(c, x, with_ls_in(a), stats, st);
}

int pml_lds_add_order_probe(const double* v, double* out, int trials, hipStream_t st) {
  if (trials <= 0) return -22;
  hipLaunchKernelGGL(lds_add_order_probe_kernel, dim3(1), dim3(64), 0, st, v, out, trials);
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
