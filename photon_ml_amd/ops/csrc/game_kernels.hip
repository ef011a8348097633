// photon_ml_amd — CDNA4 (gfx950 / MI355X) kernels for GAME scoring and the dense random-effect paths
// (row-space Gram of K7).
//
// * score_rows_kernel  — K5 fixed-effect scoring s_i = x_i . w and K6 random-effect scoring s_i = x_i . w_{e(i)}
//   over a CSR shard. 16 lanes per row (4 rows per wave64): lane-strided fp64 partial sums combined by a fixed
//   shuffle tree, so scores are bitwise reproducible. Random-effect models are entity-major CSR (eptr / sorted
//   feature ids / values, models/game.py): each lane binary-searches its feature in the row's entity segment.
//   Reference: photon-api/.../model/FixedEffectModel.scala:132-144, RandomEffectModel.scala:256-297.
// * MFMA kernels (dense GEMM-shaped work on the matrix cores, fp64 v_mfma_f64_16x16x4f64):
//   - gemm_nt_mfma_kernel — C = A B^T: back-projection of projected coefficients W P (and variances) of the
//     random projection (projector/ProjectionMatrix.scala:95-124);
// * spmm_rows_kernel — K15 forward random projection X P^T of sparse rows (ProjectionMatrix.scala:48-63).
// * downsample_kernel — K20 fixed-effect down-sampling as an on-device weight rewrite.
//
// Built with: hipcc --offload-arch=gfx950 -O3 -shared -fPIC (photon_ml_amd/ops/build.py). C ABI, ctypes.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

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

// ------------------------------------------------------------------------------------------------------------
// K5 / K6 scoring
// ------------------------------------------------------------------------------------------------------------
#define SCORE_GROUP 16                       // lanes per row
#define SCORE_THREADS 256
#define SCORE_ROWS_PER_BLOCK (SCORE_THREADS / SCORE_GROUP)

template <bool RE>
__global__ __launch_bounds__(SCORE_THREADS) void score_rows_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ col, const double* __restrict__ val,
    long long n_rows, const double* __restrict__ w, const int* __restrict__ ent,
    const long long* __restrict__ eptr, const int* __restrict__ efeat, double* __restrict__ out) {
  const long long row = (long long)blockIdx.x * SCORE_ROWS_PER_BLOCK + (threadIdx.x / SCORE_GROUP);
  const int g = threadIdx.x % SCORE_GROUP;
  double s = 0.0;
  if (row < n_rows) {
    const long long lo = indptr[row], hi = indptr[row + 1];
    long long e_lo = 0, e_hi = 0;
    bool ok = true;
    if (RE) {
      const int e = ent[row];
      if (e < 0) ok = false;
      else { e_lo = eptr[e]; e_hi = eptr[e + 1]; }
    }
    if (ok) {
      for (long long p = lo + g; p < hi; p += SCORE_GROUP) {
        const int c = col[p];
        double wv;
        if (RE) {
          long long a = e_lo, b = e_hi;         // lower bound of c in the entity's sorted feature ids
          while (a < b) {
            const long long m = (a + b) >> 1;
            if (efeat[m] < c) a = m + 1; else b = m;
          }
          wv = (a < e_hi && efeat[a] == c) ? w[a] : 0.0;
        } else {
          wv = w[c];
        }
        s += val[p] * wv;
      }
    }
  }
#pragma unroll
  for (int o = SCORE_GROUP / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, SCORE_GROUP);
  if (g == 0 && row < n_rows) out[row] = s;
}

// ------------------------------------------------------------------------------------------------------------
// MFMA: fp64 16x16x4 tiles. One wave computes a 16x16 fp64 output tile. v_mfma_f64_16x16x4_f64 fragments on
// gfx950: lane l holds A[row = l & 15][k = l >> 4] and B[k = l >> 4][col = l & 15]; accumulator i (of 4) of lane l
// holds C[row = (l >> 4) + 4 i][col = l & 15] (the f64 C/D map differs from the f32 / bf16 ones).
// ------------------------------------------------------------------------------------------------------------
typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4d mfma_f64_16x16x4(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}


// C[M x N] = A[M x K] * B[N x K]^T (all row-major fp64, leading dimensions lda / ldb / ldc). Work-group = 4 waves
// = a 32 x 32 output tile (2 x 2 wave tiles of 16 x 16); K staged through LDS in slices of 32. Grid over output
// tiles; blockIdx.x runs over N tiles fastest so neighbouring work-groups share the A panel in L2.
#define GN_T 32
#define GN_K 32
__global__ __launch_bounds__(256) void gemm_nt_mfma_kernel(int M, int N, int K, const double* __restrict__ A, int lda,
                                                            const double* __restrict__ Bm, int ldb,
                                                            double* __restrict__ C, int ldc) {
  __shared__ double sa[GN_T][GN_K + 1];
  __shared__ double sb[GN_T][GN_K + 1];
  const int tn = blockIdx.x, tm = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  v4d acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < K; k0 += GN_K) {
    __syncthreads();
    for (int idx = threadIdx.x; idx < GN_T * GN_K; idx += 256) {
      const int r = idx / GN_K, c = idx % GN_K;
      const int gr = tm * GN_T + r, gc = k0 + c;
      sa[r][c] = (gr < M && gc < K) ? A[(long long)gr * lda + gc] : 0.0;
      const int hr = tn * GN_T + r;
      sb[r][c] = (hr < N && gc < K) ? Bm[(long long)hr * ldb + gc] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GN_K; kk += 4) {
      const double a = sa[16 * wm + (lane & 15)][kk + (lane >> 4)];
      const double b = sb[16 * wn + (lane & 15)][kk + (lane >> 4)];
      acc = mfma_f64_16x16x4(a, b, acc);
    }
  }
  const int cj = tn * GN_T + 16 * wn + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ri = tm * GN_T + 16 * wm + (lane >> 4) + 4 * i;
    if (ri < M && cj < N) C[(long long)ri * ldc + cj] = acc[i];
  }
}

// K15 forward projection: Y[row][j] = sum_p val[p] * PT[col[p]][j] for a CSR X (rows) and a dense row-major
// PT [D x k] (the transposed projection matrix): one wave per row, lanes over the k outputs (strided by 64),
// non-zeros in CSR order -> deterministic. Each non-zero reads one contiguous k-row of PT (coalesced).
__global__ __launch_bounds__(256) void spmm_rows_kernel(const long long* __restrict__ indptr,
                                                         const int* __restrict__ col, const double* __restrict__ val,
                                                         long long n_rows, const double* __restrict__ PT, int k,
                                                         double* __restrict__ Y) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const long long lo = indptr[row], hi = indptr[row + 1];
  for (int j0 = 0; j0 < k; j0 += 64) {
    const int j = j0 + lane;
    double acc = 0.0;
    for (long long p = lo; p < hi; ++p) {
      const double v = val[p];
      const long long c = col[p];
      if (j < k) acc += v * PT[c * k + j];
    }
    if (j < k) Y[row * k + j] = acc;
  }
}

// K20 down-sampling (BinaryClassificationDownSampler.scala:47-68, DefaultDownSampler.scala:27-41) as a weight
// rewrite on the device: row r is kept with probability `rate` (binary tasks: every positive is kept and kept
// negatives get weight / rate), dropped rows get weight 0 — the HBM streams never change. The uniform of row r is a
// counter-based hash of (seed, global row id) (splitmix64 finaliser, top 53 bits), reproduced bit for bit by the
// host sampler (sampling/samplers.py), so CPU and GPU runs and every rank of a data-parallel job draw the same
// sample for the same row.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <typename T>
__global__ __launch_bounds__(256) void downsample_kernel(const T* __restrict__ y, const T* __restrict__ w0,
                                                          const long long* __restrict__ rowid, long long n,
                                                          unsigned long long seed, double rate, int binary,
                                                          T* __restrict__ w) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long id = rowid ? (unsigned long long)rowid[i] : (unsigned long long)i;
  const double u = (double)(splitmix64(seed ^ splitmix64(id)) >> 11) * 0x1.0p-53;
  const double wi = (double)w0[i];
  double out;
  if (binary) {
    const bool pos = (double)y[i] >= 0.5;
    out = pos ? wi : (u < rate ? wi / rate : 0.0);
  } else {
    out = u < rate ? wi : 0.0;
  }
  w[i] = (T)out;
}

// ------------------------------------------------------------------------------------------------------------
// K20 work saving: row-sampled copy of one chunk of the tiled layout (ops/tiled.py, DeviceGLMData.row_sampled).
// A down-sampled row (weight 0) adds nothing to any pass, so a fixed-effect update at rate r only needs the kept
// rows' entries (the reference trains on a physically smaller sampled RDD: DistributedOptimizationProblem.scala
// :145-160). Every work unit (forward row block / transpose item) keeps its table slot; its narrow and wide
// entries are filtered by the row keep flags and rewritten as WIDE lane-interleaved rounds in the unit's logical
// order (a filtered narrow round no longer spans < 64 keys). No sort: the filtered streams stay in unit order.
// Segments of <= CMP_SEG rounds of one unit, one wave each: pass 0 counts the kept entries per segment, the host
// turns the counts into per-unit round-aligned output starts (device cumsums) and pass 1 writes. Inside a round,
// logical entry t = 64 k + lane is placed with a ballot + popcount per k, so the copy is deterministic.
// key_is_row = 1 (transpose copy): an entry's chunk row is its key (pack >> sbits); 0 (forward copy): the unit's
// first row plus its slot (pack & smask).
// ------------------------------------------------------------------------------------------------------------
#define CMP_SEG 8
struct CmpArgs {
  const int* units;             // unit table, 6 ints per unit: ... e_lo at col_e, e_hi at col_e + 1, n_lo, n_hi at 4, 5
  int col_e, row_col;           // row_col: column of the unit's first chunk row (-1: key_is_row)
  const int* seg;               // 3 ints per segment {unit, round_lo, round_hi}; rounds [0, n_hi - n_lo) are narrow
  int nseg, sbits, key_is_row;
  const uint32_t* pack;         // wide stream (interleaved)
  const void* val;
  const uint16_t* npack;        // narrow stream (interleaved 16-bit packs), one int32 base per round
  const void* nval;
  const int* nbase;
  const unsigned char* keep;    // per chunk row: 1 = kept
  int* seg_cnt;                 // pass 0 output
  const long long* seg_first;   // pass 1: logical index (within its unit's output) of the segment's first kept entry
  const long long* unit_lo;     // pass 1: physical output start of every unit (round-aligned)
  uint32_t* opack;              // pass 1 outputs
  void* oval;
};

template <typename VT, int PASS>
__global__ __launch_bounds__(256) void tl_compact_kernel(CmpArgs a) {
  const int lane = threadIdx.x & 63;
  const int s = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (s >= a.nseg) return;                                   // wave-uniform
  const int* sg = a.seg + 3 * (long long)s;
  const int u = sg[0], r_lo = sg[1], r_hi = sg[2];
  const int* ut = a.units + 6 * (long long)u;
  const long long e_lo = ut[a.col_e];
  const int nw = ut[a.col_e + 1] - ut[a.col_e];
  const int n_lo = ut[4], nn = ut[5] - ut[4];
  const uint32_t row0 = a.row_col >= 0 ? (uint32_t)ut[a.row_col] : 0u;
  const uint32_t smask = (1u << a.sbits) - 1u;
  const VT* val = (const VT*)a.val;
  const VT* nval = (const VT*)a.nval;
  long long ob = PASS ? a.seg_first[s] : 0;
  const long long olo = PASS ? a.unit_lo[u] : 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  int cnt = 0;
  for (int r = r_lo; r < r_hi; ++r) {
    uint32_t p[4];
    VT v[4];
    bool ok[4];
    if (r < nn) {
      const long long q = (long long)n_lo + r;
      const int base = a.nbase[q];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t p16 = a.npack[q * 256 + 4 * lane + k];
        p[k] = ((uint32_t)(base + (int)(p16 >> a.sbits)) << a.sbits) | (p16 & smask);
        v[k] = nval[q * 256 + 4 * lane + k];
        ok[k] = true;
      }
    } else {
      const int w = r - nn;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ok[k] = 256 * w + 64 * k + lane < nw;
        const long long e = e_lo + 256LL * w + 4 * lane + k;
        p[k] = ok[k] ? a.pack[e] : 0u;
        v[k] = ok[k] ? val[e] : (VT)0;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t row = a.key_is_row ? (p[k] >> a.sbits) : row0 + (p[k] & smask);
      const bool kp = ok[k] && a.keep[row];
      const unsigned long long m = __ballot(kp);
      if (PASS) {
        if (kp) {
          const long long o = ob + __popcll(m & below);
          const long long ph = olo + (o & ~255LL) + ((o & 63) << 2) + ((o & 255) >> 6);
          a.opack[ph] = p[k];
          ((VT*)a.oval)[ph] = v[k];
        }
        ob += __popcll(m);
      } else {
        cnt += __popcll(m);
      }
    }
  }
  if (!PASS && lane == 0) a.seg_cnt[s] = cnt;
}


// ------------------------------------------------------------------------------------------------------------
// Per-entity Gram matrices K_e = X_e X_e^T of the row-space batch (optimization/row_space.py setup), straight
// from the block-diagonal CSR: one wave per entity of a size class (n_e <= n <= 192 rows; K zero padded to n x n).
// Row i of the entity is scattered into a dense LDS image of the entity's projected columns [cb, cb + d_e), then
// lane j takes the sparse dot product of row j with the image (row j's entries in stored order: deterministic
// fp64) and the image is cleared entry by entry. Rows must hold distinct columns (canonical CSR; checked on the
// host). Replaces 2 x n full passes of the GLM kernels over the whole coordinate (one indicator column per pass).
// ------------------------------------------------------------------------------------------------------------
// S rows per scatter round (template): rows i0 .. i0 + S - 1 go into S interleaved image slots (img[c S + s]), and
// one walk over row j's entries feeds S accumulators -- S times fewer walks (global reads + dependent chains) than
// one row per round, the same fma sequence per K entry (bitwise equal for every S).
// STAGE: the entity's entries (local column as uint16, value) and row offsets are first copied into LDS with
// coalesced whole-wave loads; the per-lane walks over row j then read LDS instead of issuing one uncoalesced global
// load per entry (64 lanes on 64 different rows) -- the dependent chain of a walk is LDS-latency bound, not
// HBM-latency bound. Same fma sequence, bitwise equal to the unstaged walk.
template <int S, bool STAGE>
__global__ __launch_bounds__(64) void seg_gram_kernel(int B, int n, int dmax, const long long* __restrict__ ents,
                                                      const long long* __restrict__ row_ptr,
                                                      const long long* __restrict__ col_ptr,
                                                      const long long* __restrict__ nip,
                                                      const long long* __restrict__ pos,
                                                      const double* __restrict__ val, double* __restrict__ K) {
  extern __shared__ double img[];
  const int lane = threadIdx.x;
  const long long b = blockIdx.x;
  if (b >= B) return;
  const long long e = ents[b];
  const long long r0 = row_ptr[e];
  const int ne = (int)(row_ptr[e + 1] - r0);
  const long long cb = col_ptr[e];
  const int de = (int)(col_ptr[e + 1] - cb);
  const long long e0 = nip[r0];
  const int enz = (int)(nip[r0 + ne] - e0);
  // staged layout after the image: values [enz] doubles, local columns [enz] uint16, row offsets [ne + 1] int
  double* sval = img + (size_t)dmax * S;
  unsigned short* scol = (unsigned short*)(sval + enz);
  int* sptr = (int*)(scol + ((enz + 3) & ~3));
  for (int c = lane; c < de * S; c += 64) img[c] = 0.0;
  if (STAGE) {
    for (int t = lane; t < enz; t += 64) {
      sval[t] = val[e0 + t];
      scol[t] = (unsigned short)(pos[e0 + t] - cb);
    }
    for (int i = lane; i <= ne; i += 64) sptr[i] = (int)(nip[r0 + i] - e0);
  }
  __syncthreads();
  double* Kb = K + b * (long long)n * n;
  for (int i0 = 0; i0 < ne; i0 += S) {
    const int ns = ne - i0 < S ? ne - i0 : S;
    for (int s = 0; s < ns; ++s) {
      if (STAGE) {
        const int ib = sptr[i0 + s], ie = sptr[i0 + s + 1];
        for (int t = ib + lane; t < ie; t += 64) img[(int)scol[t] * S + s] = sval[t];
      } else {
        const long long ib = nip[r0 + i0 + s], ie = nip[r0 + i0 + s + 1];
        for (long long t = ib + lane; t < ie; t += 64) img[(pos[t] - cb) * S + s] = val[t];
      }
    }
    __syncthreads();
    // lane takes rows j = lane, lane + 64, lane + 128 (n <= 192)
    for (int j = lane; j < n; j += 64) {
      double acc[S];
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = 0.0;
      if (j < ne) {
        if (STAGE) {
          const int jb = sptr[j], je = sptr[j + 1];
          for (int t = jb; t < je; ++t) {
            const double v = sval[t];
            const double* im = img + (int)scol[t] * S;
#pragma unroll
            for (int s = 0; s < S; ++s) acc[s] = fma(v, im[s], acc[s]);
          }
        } else {
          const long long jb = nip[r0 + j], je = nip[r0 + j + 1];
          for (long long t = jb; t < je; ++t) {
            const double v = val[t];
            const double* im = img + (pos[t] - cb) * S;
#pragma unroll
            for (int s = 0; s < S; ++s) acc[s] = fma(v, im[s], acc[s]);
          }
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (s < ns) Kb[(long long)j * n + i0 + s] = acc[s];
    }
    __syncthreads();
    for (int s = 0; s < ns; ++s) {
      if (STAGE) {
        const int ib = sptr[i0 + s], ie = sptr[i0 + s + 1];
        for (int t = ib + lane; t < ie; t += 64) img[(int)scol[t] * S + s] = 0.0;
      } else {
        const long long ib = nip[r0 + i0 + s], ie = nip[r0 + i0 + s + 1];
        for (long long t = ib + lane; t < ie; t += 64) img[(pos[t] - cb) * S + s] = 0.0;
      }
    }
    __syncthreads();
  }
  for (int i = ne; i < n; ++i)
    for (int j = lane; j < n; j += 64) Kb[(long long)j * n + i] = 0.0;
}

// Batched Cholesky of the row-space Gram matrices (replaces torch.linalg.cholesky_ex = rocSOLVER dpotf2: 48
// launches per class set and a one-off library initialisation on the cold path). One wave per problem, the lower
// triangle packed in LDS (n (n + 1) / 2 doubles: <= 148 KB at n = 192), left-looking: column j's entries are dot
// products of row prefixes, lanes over rows i >= j. Rows i >= nv[b] (padding slots) are the identity. Writes the
// full n x n factor (upper triangle zero) over K; info[b] = 0, or j + 1 for the first non-positive / non-finite
// pivot (then the factor is not used).
__global__ __launch_bounds__(64) void batched_chol_kernel(int B, int n, const long long* __restrict__ nv,
                                                          double* __restrict__ K, int* __restrict__ info) {
  extern __shared__ double Lp[];
  const int lane = threadIdx.x;
  const long long b = blockIdx.x;
  if (b >= B) return;
  const int m = (int)nv[b];
  double* Kb = K + b * (long long)n * n;
  for (int i = lane; i < n; i += 64)
    for (int k = 0; k <= i; ++k)
      Lp[i * (i + 1) / 2 + k] = (i < m && k < m) ? Kb[(long long)i * n + k] : (i == k ? 1.0 : 0.0);
  __syncthreads();
  int bad = 0;
  for (int j = 0; j < m && !bad; ++j) {
    const int rj = j * (j + 1) / 2;
    double djj = Lp[rj + j];
    for (int k = 0; k < j; ++k) djj = fma(-Lp[rj + k], Lp[rj + k], djj);
    __syncthreads();
    if (!(djj > 0.0) || !isfinite(djj)) { bad = j + 1; break; }
    const double ljj = sqrt(djj);
    for (int i = j + 1 + lane; i < m; i += 64) {
      const int ri = i * (i + 1) / 2;
      double a = Lp[ri + j];
      for (int k = 0; k < j; ++k) a = fma(-Lp[ri + k], Lp[rj + k], a);
      Lp[ri + j] = a / ljj;
    }
    if (lane == 0) Lp[rj + j] = ljj;
    __syncthreads();
  }
  if (lane == 0) info[b] = bad;
  for (int i = lane; i < n; i += 64)
    for (int k = 0; k < n; ++k) Kb[(long long)i * n + k] = k <= i ? Lp[i * (i + 1) / 2 + k] : 0.0;
}

// Row-space back-map w_e = X_e^T r_e for the entities ents[B] (random-effect model materialisation,
// optimization/row_space.py to_primal): one wave per entity, the entity's projected columns accumulated in LDS
// (d_e doubles), rows in order and the entries of one row on distinct lanes with distinct columns, so every LDS
// address is updated in a fixed order (deterministic) and no two lanes of one instruction collide. Reads only the
// handled entities' rows (the shard-wide transpose pass read every entity's).
// PT: int64 or int32 packed positions (int32 when the packed vector has < 2^31 coefficients: 4 bytes less per entry
// of a bandwidth-bound pass)
template <typename PT>
__global__ __launch_bounds__(64) void rs_primal_kernel(const long long* __restrict__ ents,
                                                       const long long* __restrict__ row_ptr,
                                                       const long long* __restrict__ col_ptr,
                                                       const long long* __restrict__ nip,
                                                       const PT* __restrict__ pos,
                                                       const double* __restrict__ val, const double* __restrict__ r,
                                                       double* __restrict__ W) {
  extern __shared__ double acc[];
  const int lane = threadIdx.x;
  const long long e = ents[blockIdx.x];
  const long long r0 = row_ptr[e], r1 = row_ptr[e + 1], c0 = col_ptr[e];
  const int d = (int)(col_ptr[e + 1] - c0);
  for (int j = lane; j < d; j += 64) acc[j] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (long long i = r0; i < r1; ++i) {
    const double a = r[i];
    const long long k0 = nip[i], k1 = nip[i + 1];
    for (long long k = k0 + lane; k < k1; k += 64) {
      const int c = (int)((long long)pos[k] - c0);
      acc[c] += a * val[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  for (int j = lane; j < d; j += 64) W[c0 + j] = acc[j];
}

// ---------------------------------------------------------------------------------------------------------------
// Histogram of integer keys (torch.bincount) for inputs with very hot keys: the fixed-effect relabel counts 775M
// column ids of which one (the intercept) occurs in EVERY row and a Zipf head in most, so plain global atomics
// serialise on a few addresses (torch's kernelHistogram1D: 443 ms at GAME config 5). Each workgroup aggregates its
// slice in an LDS open-addressing table (HIST_SLOTS keys, linear probing, HIST_PROBES tries) and flushes one global
// atomic per distinct key it holds; keys that find no slot go straight to global atomics (they are the rare ones).
// Integer counts: the result does not depend on the order of the atomics.
#define HIST_SLOTS 4096
#define HIST_PROBES 8
#define HIST_THREADS 256
template <typename KT>
__global__ __launch_bounds__(HIST_THREADS) void key_hist_kernel(const KT* __restrict__ keys, long long n,
                                                                long long per_block, long long nbins,
                                                                unsigned long long* __restrict__ counts) {
  __shared__ int s_key[HIST_SLOTS];
  __shared__ unsigned int s_cnt[HIST_SLOTS];
  for (int i = threadIdx.x; i < HIST_SLOTS; i += HIST_THREADS) { s_key[i] = -1; s_cnt[i] = 0; }
  __syncthreads();
  const long long a = (long long)blockIdx.x * per_block;
  const long long b = a + per_block < n ? a + per_block : n;
  for (long long i = a + threadIdx.x; i < b; i += HIST_THREADS) {
    const long long k = (long long)keys[i];
    if (k < 0 || k >= nbins) continue;                       // the wrapper validates; never index out of range
    bool done = false;
    if (k < 0x7fffffffLL) {
      const int ki = (int)k;
      unsigned int h = ((unsigned int)ki * 2654435761u) >> (32 - 12);
      for (int p = 0; p < HIST_PROBES && !done; ++p) {
        const int s = (int)((h + (unsigned int)p) & (HIST_SLOTS - 1));
        int cur = s_key[s];
        if (cur == -1) cur = atomicCAS(&s_key[s], -1, ki) == -1 ? ki : s_key[s];
        if (cur == ki) { atomicAdd(&s_cnt[s], 1u); done = true; }
      }
    }
    if (!done) atomicAdd(&counts[k], 1ULL);
  }
  __syncthreads();
  for (int s = threadIdx.x; s < HIST_SLOTS; s += HIST_THREADS) {
    const int k = s_key[s];
    if (k >= 0 && s_cnt[s]) atomicAdd(&counts[k], (unsigned long long)s_cnt[s]);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Row gather of a CSR into a new CSR (random-effect solver setup: the fused primal batch's rows, the row-space
// back-map's compact copy). Row r of the output = row rows[r] of the input, starting at optr[r] with
// optr[r + 1] - optr[r] >= its length slots (extra slots zero-filled: the lean kernel's quad padding); columns minus
// cbase[r] (entity-local) when cbase is given, stored as CT (int16 / int64). One wave per row, coalesced copies:
// replaces a chain of torch repeat_interleave / gather / scatter passes over every non-zero.
template <typename CT>
__global__ __launch_bounds__(256) void csr_gather_rows_kernel(const long long* __restrict__ nip,
                                                              const long long* __restrict__ pos,
                                                              const double* __restrict__ val,
                                                              const long long* __restrict__ rows, long long nr,
                                                              const long long* __restrict__ optr,
                                                              const long long* __restrict__ cbase,
                                                              CT* __restrict__ ocol, double* __restrict__ oval) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= nr) return;
  const long long src = nip[rows[r]], len = nip[rows[r] + 1] - src;
  const long long dst = optr[r], dlen = optr[r + 1] - dst;
  const long long base = cbase != nullptr ? cbase[r] : 0;
  for (long long t = lane; t < dlen; t += 64) {
    if (t < len) {
      ocol[dst + t] = (CT)(pos[src + t] - base);
      oval[dst + t] = val[src + t];
    } else {
      ocol[dst + t] = (CT)0;
      oval[dst + t] = 0.0;
    }
  }
}

extern "C" {

const char* pml_build_id() { return pml_build_stamp + 13; }

int pml_downsample(int f64, const void* y, const void* w0, const long long* rowid, long long n,
                   unsigned long long seed, double rate, int binary, void* w, void* stream) {
  if (n <= 0) return 0;
  const long long blocks = (n + 255) / 256;
  if (blocks > 0x7fffffffLL) return -22;
  if (f64)
    hipLaunchKernelGGL(downsample_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const double*)y, (const double*)w0, rowid, n, seed, rate, binary, (double*)w);
  else
    hipLaunchKernelGGL(downsample_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const float*)y, (const float*)w0, rowid, n, seed, rate, binary, (float*)w);
  LAUNCH_CHECK();
  return 0;
}

// pass 0: count, 1: write; vbytes = sizeof(value) (bf16 2, fp32 4, fp64 8)
int pml_tl_compact(int pass, int vbytes, const CmpArgs* a, void* stream) {
  if (a->nseg <= 0) return 0;
  const dim3 grid((unsigned)((a->nseg + 3) / 4)), blk(256);
  hipStream_t st = (hipStream_t)stream;
#define CMP_LAUNCH(VT)                                                              \
  do {                                                                              \
    if (pass) hipLaunchKernelGGL((tl_compact_kernel<VT, 1>), grid, blk, 0, st, *a); \
    else hipLaunchKernelGGL((tl_compact_kernel<VT, 0>), grid, blk, 0, st, *a);      \
  } while (0)
  if (vbytes == 2) CMP_LAUNCH(unsigned short);
  else if (vbytes == 4) CMP_LAUNCH(unsigned int);
  else if (vbytes == 8) CMP_LAUNCH(unsigned long long);
  else return -22;
#undef CMP_LAUNCH
  LAUNCH_CHECK();
  return 0;
}

int pml_spmm_rows(const long long* indptr, const int* col, const double* val, long long n_rows, const double* PT,
                  int k, double* Y, void* stream) {
  if (n_rows <= 0 || k <= 0) return 0;
  const long long blocks = (n_rows + 3) / 4;
  if (blocks > 0x7fffffffLL) return -22;
  hipLaunchKernelGGL(spmm_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, indptr, col, val,
                     n_rows, PT, k, Y);
  LAUNCH_CHECK();
  return 0;
}

int pml_score_rows(const long long* indptr, const int* col, const double* val, long long n_rows, const double* w,
                   const int* ent, const long long* eptr, const int* efeat, double* out, void* stream) {
  if (n_rows <= 0) return 0;
  const long long blocks = (n_rows + SCORE_ROWS_PER_BLOCK - 1) / SCORE_ROWS_PER_BLOCK;
  if (blocks > 0x7fffffffLL) return -22;
  if (ent) {
    hipLaunchKernelGGL(score_rows_kernel<true>, dim3((unsigned)blocks), dim3(SCORE_THREADS), 0, (hipStream_t)stream,
                       indptr, col, val, n_rows, w, ent, eptr, efeat, out);
  } else {
    hipLaunchKernelGGL(score_rows_kernel<false>, dim3((unsigned)blocks), dim3(SCORE_THREADS), 0,
                       (hipStream_t)stream, indptr, col, val, n_rows, w, ent, eptr, efeat, out);
  }
  LAUNCH_CHECK();
  return 0;
}


int pml_gemm_nt(int M, int N, int K, const double* A, int lda, const double* Bm, int ldb, double* C, int ldc,
                void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 0) return -22;
  dim3 grid((N + GN_T - 1) / GN_T, (M + GN_T - 1) / GN_T);
  hipLaunchKernelGGL(gemm_nt_mfma_kernel, grid, dim3(256), 0, (hipStream_t)stream, M, N, K, A, lda, Bm, ldb, C, ldc);
  LAUNCH_CHECK();
  return 0;
}


static int g_seg_gram_s = 0;   // rows per scatter round of seg_gram_kernel (0: by LDS size; A/B: pml_seg_gram_set_s)
void pml_seg_gram_set_s(int s) { g_seg_gram_s = (s == 1 || s == 2 || s == 4 || s == 8) ? s : 0; }

// K [B, n, n] for the entities ents[B]; dmax = max projected columns of those entities (LDS image size); maxnnz = max
// non-zeros of one of those entities (> 0: stage the entries in LDS when they fit, see seg_gram_kernel STAGE).
int pml_seg_gram(int B, int n, int dmax, long long maxnnz, const long long* ents, const long long* row_ptr,
                 const long long* col_ptr, const long long* nip, const long long* pos, const double* val, double* K,
                 void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 192 || dmax < 0 || (size_t)dmax * sizeof(double) > 160 * 1024) return -22;
  // rows per scatter round: as many as keep the image <= 32 KB (>= 5 one-wave workgroups per CU)
  const size_t d8 = (size_t)std::max(dmax, 1) * sizeof(double);
  const int S = g_seg_gram_s > 0 ? g_seg_gram_s : (d8 * 8 <= 32768 ? 8 : d8 * 4 <= 32768 ? 4 : d8 * 2 <= 32768 ? 2 : 1);
  const size_t img = d8 * (size_t)S;
  const size_t stage = maxnnz > 0 ? (size_t)maxnnz * 10 + 8 + (size_t)(n + 1) * 4 + 16 : 0;
  const bool staged = maxnnz > 0 && img + stage <= 64 * 1024;
  const size_t lds = staged ? img + stage : img;
  if (lds > 160 * 1024) return -22;
  hipStream_t st = (hipStream_t)stream;
#define SEG_GRAM_LAUNCH(SS)                                                                                       \
  do {                                                                                                           \
    if (staged)                                                                                                  \
      hipLaunchKernelGGL((seg_gram_kernel<SS, true>), dim3((unsigned)B), dim3(64), lds, st, B, n, std::max(dmax, 1), \
                         ents, row_ptr, col_ptr, nip, pos, val, K);                                              \
    else                                                                                                         \
      hipLaunchKernelGGL((seg_gram_kernel<SS, false>), dim3((unsigned)B), dim3(64), lds, st, B, n, std::max(dmax, 1), \
                         ents, row_ptr, col_ptr, nip, pos, val, K);                                              \
  } while (0)
  if (S == 8) SEG_GRAM_LAUNCH(8);
  else if (S == 4) SEG_GRAM_LAUNCH(4);
  else if (S == 2) SEG_GRAM_LAUNCH(2);
  else SEG_GRAM_LAUNCH(1);
#undef SEG_GRAM_LAUNCH
  LAUNCH_CHECK();
  return 0;
}

// In-place Cholesky of K [B, n, n] (n <= 192); nv[b] = valid rows of problem b (the rest: identity); info[B].
int pml_batched_chol(int B, int n, const long long* nv, double* K, int* info, void* stream) {
  if (B <= 0) return 0;
  if (n < 1 || n > 192) return -22;
  const size_t lds = (size_t)n * (n + 1) / 2 * sizeof(double);
  hipLaunchKernelGGL(batched_chol_kernel, dim3((unsigned)B), dim3(64), lds, (hipStream_t)stream, B, n, nv, K, info);
  LAUNCH_CHECK();
  return 0;
}

// W (packed projected coefficients) of the entities ents[B] = X_e^T r over their rows; dmax = max projected columns
// of those entities (LDS per wave). Other entities' coefficients are left untouched.
// pos32: positions are int32 (else int64).
int pml_rs_primal(int B, int dmax, const long long* ents, const long long* row_ptr, const long long* col_ptr,
                  const long long* nip, const void* pos, const double* val, const double* r, double* W,
                  void* stream, int pos32) {
  if (B <= 0) return 0;
  if (dmax < 0 || (size_t)dmax * sizeof(double) > 64 * 1024) return -22;
  const size_t lds = (size_t)std::max(dmax, 1) * sizeof(double);
  if (pos32)
    hipLaunchKernelGGL(rs_primal_kernel<int>, dim3((unsigned)B), dim3(64), lds, (hipStream_t)stream, ents, row_ptr,
                       col_ptr, nip, (const int*)pos, val, r, W);
  else
    hipLaunchKernelGGL(rs_primal_kernel<long long>, dim3((unsigned)B), dim3(64), lds, (hipStream_t)stream, ents,
                       row_ptr, col_ptr, nip, (const long long*)pos, val, r, W);
  LAUNCH_CHECK();
  return 0;
}
// counts[nbins] += histogram of keys[n] (int32 if k32 else int64); counts must be zeroed by the caller
int pml_key_hist(int k32, const void* keys, long long n, long long nbins, unsigned long long* counts, void* stream) {
  if (n <= 0) return 0;
  const long long per_block = 1 << 16;
  const long long blocks = (n + per_block - 1) / per_block;
  if (blocks > 0x7fffffffLL) return -22;
  if (k32)
    hipLaunchKernelGGL(key_hist_kernel<int>, dim3((unsigned)blocks), dim3(HIST_THREADS), 0, (hipStream_t)stream,
                       (const int*)keys, n, per_block, nbins, counts);
  else
    hipLaunchKernelGGL(key_hist_kernel<long long>, dim3((unsigned)blocks), dim3(HIST_THREADS), 0,
                       (hipStream_t)stream, (const long long*)keys, n, per_block, nbins, counts);
  LAUNCH_CHECK();
  return 0;
}

// out (col as int16 if c16 else int64, val fp64) = rows[nr] of (nip, pos, val) at optr, minus cbase (may be null)
int pml_csr_gather_rows(int c16, const long long* nip, const long long* pos, const double* val, const long long* rows,
                        long long nr, const long long* optr, const long long* cbase, void* ocol, double* oval,
                        void* stream) {
  if (nr <= 0) return 0;
  const long long blocks = (nr + 3) / 4;
  if (blocks > 0x7fffffffLL) return -22;
  if (c16)
    hipLaunchKernelGGL(csr_gather_rows_kernel<short>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, nip,
                       pos, val, rows, nr, optr, cbase, (short*)ocol, oval);
  else
    hipLaunchKernelGGL(csr_gather_rows_kernel<long long>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       nip, pos, val, rows, nr, optr, cbase, (long long*)ocol, oval);
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
