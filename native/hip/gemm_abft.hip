// ABFT (algorithm-based fault tolerance) check of a validator GEMM: every output element is covered,
// and a wrong result is localised to the output tile that holds it.
//
//   C[M,N] (bf16) = A[M,K] * Bt[N,K]^T, operands bf16 or fp8 e4m3fn (K-major), fp32 accumulation.
//
// The reference's only GPU check is CUDA-samples vectorAdd, which verifies every element it computes
// on the host (validator/cuda-workload-validation.yaml:15-25). A GEMM's output cannot
// be recomputed element by element at validator speed, but its tile sums can (Huang & Abraham's
// checksum GEMM, here per output tile):
//
//   row check     for every row m and N-strip j (the TN columns of tile column j):
//                   sum_{n in j} C[m,n]  ==  sum_k A[m,k] * WB[j][k],   WB[j][k] = sum_{n in j} Bt[n,k]
//   column check  for every column n and M-strip i (the TM rows of tile row i):
//                   sum_{m in i} C[m,n]  ==  sum_k WA[i][k] * Bt[n,k],  WA[i][k] = sum_{m in i} A[m,k]
//
// Both sides are fp32 on the vector ALUs -- no matrix core, no hardware fp8 converter: the check
// shares no datapath with the kernel it checks. A failing row sum names tile (m / TM, j), a failing
// column sum tile (i, n / TN); every element sits in one row sum and one column sum, so
// checked_fraction is 1.
//
// Tolerance per sum: the output is bf16, rounded to nearest from fp32, so each element carries an
// error of at most half its ulp; for the s elements of a sum, Hoeffding bounds
//   P(|sum of errors| >= t) <= 2 exp(-2 t^2 / sum ulp_i^2),
// which is <= 1e-15 at t = 4.2 sqrt(sum ulp_i^2): tol = 4.5 sqrt(U) with U = sum of ulp^2 of the
// output elements (from their exponents) -- plus 2^-18 of sum_k |x_k w_k| for the two fp32
// accumulation orders. At 8192^3 (uniform [-1,1) operands, |C| ~ 30) a sum of 256 elements tolerates
// ~9, against sums of ~500: one element off by more than ~9 (an exponent or high-mantissa bit flip,
// a lost MFMA, a stale or unwritten tile) fails; a flip of the lowest mantissa bits of one element is
// below the output's own rounding noise and is not seen -- no checksum over rounded outputs can.
// A non-finite element fails its sums (the comparison is !(d <= tol)).
//
// Cost at 8192^3 bf16 (one check): strip sums of A and Bt (2 x 128 MiB read), two fp32 GEMV-like
// products (2 x 2.1 G multiply-adds), one pass over C (128 MiB), the compare -- well under a
// millisecond next to a probe of 100+ ms (amd-gemm-validate prints check_ms and probe_ms).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>

namespace {

constexpr int ABFT_THREADS = 256;

// OCP e4m3fn -> fp32 in software (the check must not share the fp8 converter with the GEMM's fill).
__device__ __forceinline__ float abft_ld(const uint8_t* p, size_t i) {
  const uint32_t v = p[i];
  const int e = (v >> 3) & 15, m = v & 7;
  float f = e ? __builtin_amdgcn_ldexpf((float)(8 + m), e - 10) : __builtin_amdgcn_ldexpf((float)m, -9);
  if ((v & 0x7F) == 0x7F) f = __builtin_nanf("");
  return (v & 0x80) ? -f : f;
}
__device__ __forceinline__ float abft_ld(const __bf16* p, size_t i) { return (float)p[i]; }

// W[t][k] = sum of X[r][k] over the rows r of strip t (S rows), Wabs the same of |X[r][k]|.
// grid (ceil(K / 256), strips); one column per thread, rows walked in order (coalesced across k).
template <class T>
__global__ void __launch_bounds__(ABFT_THREADS)
abft_strip_sums(const T* __restrict__ X, int R, int K, int S, float* __restrict__ W, float* __restrict__ Wabs) {
  const int k = blockIdx.x * ABFT_THREADS + threadIdx.x;
  if (k >= K) return;
  const int t = blockIdx.y;
  const int r0 = t * S, r1 = min(R, r0 + S);
  float s = 0.f, a = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) {
    const float v = abft_ld(X, (size_t)r * K + k);
    s += v;
    a += fabsf(v);
  }
  W[(size_t)t * K + k] = s;
  Wabs[(size_t)t * K + k] = a;
}

// 8 consecutive elements X[i..i+7] as fp32: one 16-byte (bf16) / 8-byte (fp8) load when `vec`
// (in bounds and aligned), else guarded scalar loads up to `n` elements.
__device__ __forceinline__ void abft_ld8(const __bf16* p, size_t i, int n, bool vec, float* out) {
  if (vec) {
    const uint4 q = *(const uint4*)(p + i);
    const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      out[2 * e] = __uint_as_float(u[e] << 16);
      out[2 * e + 1] = __uint_as_float(u[e] & 0xFFFF0000u);
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = e < n ? abft_ld(p, i + e) : 0.f;
}
__device__ __forceinline__ void abft_ld8(const uint8_t* p, size_t i, int n, bool vec, float* out) {
  if (vec) {
    const uint2 q = *(const uint2*)(p + i);
    const uint8_t b[8] = {(uint8_t)q.x, (uint8_t)(q.x >> 8), (uint8_t)(q.x >> 16), (uint8_t)(q.x >> 24),
                          (uint8_t)q.y, (uint8_t)(q.y >> 8), (uint8_t)(q.y >> 16), (uint8_t)(q.y >> 24)};
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = abft_ld(b, e);
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = e < n ? abft_ld(p, i + e) : 0.f;
}

// E[z][r][j] = sum over K-slice z of X[r][k] W[j][k], Eabs the same of |X[r][k] W[j][k]|, for r < R,
// j < J. A 32-row x 32-strip block of 256 threads: thread (ty, tx) owns row tx and strips 4ty..4ty+3;
// the block's K-slice (blockIdx.z, `kper` long, a multiple of 64) in chunks of 64 staged through LDS
// by one 8-element vector load per thread and operand (X as fp32 [row][k], padded; W transposed
// [k][strip], so a thread's four strips are one 16-byte broadcast read). K is sliced so the grid has
// ~1024 blocks (a 32-strip check of 8192 rows is 256 blocks, one wave per SIMD and a global-load wait
// per chunk: 1 ms; sliced, 4 blocks per CU hide each other's loads); the compare sums the slices in
// order, so the result does not depend on scheduling.
constexpr int EX_R = 32, EX_J = 32, EX_KC = 64;

template <class T>
__global__ void __launch_bounds__(ABFT_THREADS)
abft_expect(const T* __restrict__ X, int R, int K, const float* __restrict__ W, int J, int kper,
            float* __restrict__ E, float* __restrict__ Eabs) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float xs[EX_R][EX_KC + 1];
  __shared__ __attribute__((aligned(16))) float ws[EX_KC][EX_J + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 31, ty = tid >> 5;
  const int r0 = blockIdx.x * EX_R, j0 = blockIdx.y * EX_J;
  const int kb = blockIdx.z * kper, ke = min(K, kb + kper);
  const int lr = tid >> 3, lk = (tid & 7) * 8;      // staging: row / strip lr, elements lk..lk+7
  const bool xvec = (K & 7) == 0, wvec = (K & 3) == 0;
  f4 acc = {0.f, 0.f, 0.f, 0.f}, aab = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += EX_KC) {
    {
      float v[8];
      const int k = k0 + lk, n = min(8, ke - k);
      if (r0 + lr < R && n > 0) abft_ld8(X, (size_t)(r0 + lr) * K + k, n, xvec && n == 8, v);
      else
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) xs[lr][lk + e] = v[e];
    }
    {
      float v[8];
      const int k = k0 + lk, n = min(8, ke - k);
      const float* w = W + (size_t)(j0 + lr) * K + k;
      if (j0 + lr < J && n == 8 && wvec) {
        const f4 a = *(const f4*)w, b = *(const f4*)(w + 4);
        for (int e = 0; e < 4; ++e) v[e] = a[e], v[e + 4] = b[e];
      } else {
        for (int e = 0; e < 8; ++e) v[e] = (j0 + lr < J && e < n) ? w[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ws[lk + e][lr] = v[e];
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < EX_KC; ++kk) {
      const float x = xs[tx][kk];
      const f4 w = *(const f4*)&ws[kk][ty * 4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q] = fmaf(x, w[q], acc[q]);
        aab[q] = fmaf(fabsf(x), fabsf(w[q]), aab[q]);
      }
    }
    __syncthreads();
  }
  const int r = r0 + tx;
  if (r >= R) return;
  const size_t base = ((size_t)blockIdx.z * R + r) * J;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = j0 + ty * 4 + q;
    if (j < J) {
      E[base + j] = acc[q];
      Eabs[base + j] = aab[q];
    }
  }
}

// The K slicing of an expect launch: slices of a multiple of 64 elements, enough of them for ~1024
// blocks, at most 8.
struct ExSplit {
  int kper, slices;
};
ExSplit ex_split(int R, int J, int K) {
  const long long blocks = (long long)((R + EX_R - 1) / EX_R) * ((J + EX_J - 1) / EX_J);
  int want = (int)std::max(1LL, std::min(8LL, 1024 / std::max(1LL, blocks)));
  int kper = (K + want - 1) / want;
  kper = (kper + EX_KC - 1) / EX_KC * EX_KC;
  return {kper, (K + kper - 1) / kper};
}

// ulp(x)^2 of a bf16 from its bits: 2^(2(e - 134)) for biased exponent e (7 stored mantissa bits),
// the subnormal ulp for e = 0; 0 for Inf/NaN (the sum itself is non-finite then).
__device__ __forceinline__ float bf16_ulp2(uint32_t bits) {
  const int e = (bits >> 7) & 0xFF;
  if (e == 0xFF) return 0.f;
  return __builtin_amdgcn_ldexpf(1.f, 2 * (e > 0 ? e : 1) - 268);
}

// One pass over C: row sums per N-strip (Srow / Urow [m][j], j = n / TN) and column sums per M-strip
// (ScolT / UcolT [n][i], i = m / TM), U = sum of ulp^2. grid (ceil(N / 512), ceil(M / TM)), 4 waves:
// lane l of every wave holds columns 8l..8l+7 of the block's 512, wave w rows w, w+4, ... of strip i.
// G = TN / 8 lanes share an N-strip: their row partials meet by xor-shuffles. The column partials
// of the 4 waves meet in LDS, summed in wave order (deterministic).
template <int G>
__global__ void __launch_bounds__(ABFT_THREADS)
abft_c_sums(const __bf16* __restrict__ C, int M, int N, int TM, int J, int I, float* __restrict__ Srow,
            float* __restrict__ Urow, float* __restrict__ ScolT, float* __restrict__ UcolT) {
  __shared__ float red[2][4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int i = blockIdx.y;
  const int r0 = i * TM, r1 = min(M, r0 + TM);
  const uint16_t* Cb = (const uint16_t*)C;
  float cs[8], cu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cu[e] = 0.f;
  for (int r = r0 + w; r < r1; r += 4) {
    uint32_t bits[8];
    if (c0 + 8 <= N && (N & 7) == 0) {
      const uint4 q = *(const uint4*)(Cb + (size_t)r * N + c0);
      const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bits[2 * e] = u[e] & 0xFFFF;
        bits[2 * e + 1] = u[e] >> 16;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bits[e] = c0 + e < N ? Cb[(size_t)r * N + c0 + e] : 0u;
    }
    float rs = 0.f, ru = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = __uint_as_float(bits[e] << 16);
      const float u = bf16_ulp2(bits[e]);
      rs += v;
      ru += u;
      cs[e] += v;
      cu[e] += u;
    }
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
      rs += __shfl_xor(rs, off);
      ru += __shfl_xor(ru, off);
    }
    if ((lane & (G - 1)) == 0 && c0 < N) {
      const int j = c0 / (8 * G);
      Srow[(size_t)r * J + j] = rs;
      Urow[(size_t)r * J + j] = ru;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][w][lane * 8 + e] = cs[e];
    red[1][w][lane * 8 + e] = cu[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += ABFT_THREADS) {
    const int n = blockIdx.x * 512 + c;
    if (n >= N) continue;
    ScolT[(size_t)n * I + i] = ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    UcolT[(size_t)n * I + i] = ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
  }
}

// Compare one check ([R][J] sums against expectations) and flag the tiles of the failing sums. Row
// check (col = 0): r = m, j = the tile column; column check (col = 1): r = n, j = the tile row.
// `worst` (as int bits of a non-negative float) gets the largest |S - E| / tol of the grid, one atomic
// per wave; a failing sum also sets bit (1 << col) of its tile's flag.
__global__ void __launch_bounds__(ABFT_THREADS)
abft_compare(const float* __restrict__ S, const float* __restrict__ U, const float* __restrict__ E,
             const float* __restrict__ Eabs, int slices, int R, int J, int rows_per_tile, int tiles_n, int col,
             float k_sigma, float rel_slack, int* __restrict__ flags, int* __restrict__ worst) {
  const size_t idx = (size_t)blockIdx.x * ABFT_THREADS + threadIdx.x;
  float ratio = 0.f;
  if (idx < (size_t)R * J) {
    const int r = (int)(idx / J), j = (int)(idx % J);
    float e = 0.f, ea = 0.f;
    for (int z = 0; z < slices; ++z) {
      e += E[(size_t)z * R * J + idx];
      ea += Eabs[(size_t)z * R * J + idx];
    }
    const float d = fabsf(S[idx] - e);
    const float tol = k_sigma * sqrtf(U[idx]) + rel_slack * ea + 1e-30f;
    const bool bad = !(d <= tol);
    ratio = bad && !(d == d && d < __builtin_inff()) ? __builtin_inff() : d / tol;
    if (bad) {
      const int t = col ? j * tiles_n + r / rows_per_tile : (r / rows_per_tile) * tiles_n + j;
      atomicOr(&flags[t], 1 << col);
    }
  }
  for (int off = 32; off > 0; off >>= 1) ratio = fmaxf(ratio, __shfl_xor(ratio, off));
  if ((threadIdx.x & 63) == 0) atomicMax(worst, __float_as_int(ratio));
}

// fp32 reference of sampled output rows (the validator's second opinion next to the checksums, and
// ops.gemm.reference_rows): out[i][n] = sum_k A[rows[i]][k] Bt[n][k] is the expectation product above
// with X = Bt and the gathered A rows as W -- vector-ALU fp32, software fp8 decode, no matrix core.
// (A thread-per-column kernel read Bt with a stride of K per lane: 20 ms for 32 rows at 8192^3.)
template <class T>
__global__ void __launch_bounds__(ABFT_THREADS)
gather_rows_f32(const T* __restrict__ A, const int* __restrict__ rows, int nrows, int K, float* __restrict__ out) {
  const int i = blockIdx.y;
  for (int k = blockIdx.x * ABFT_THREADS + threadIdx.x; k < K; k += gridDim.x * ABFT_THREADS)
    out[(size_t)i * K + k] = abft_ld(A, (size_t)rows[i] * K + k);
}

// out[i][n] = sum of the slices E[z][n][i]
__global__ void __launch_bounds__(ABFT_THREADS)
ref_rows_finish(const float* __restrict__ E, int slices, int N, int nrows, float* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * ABFT_THREADS + threadIdx.x;
  if (idx >= (size_t)N * nrows) return;
  const int n = (int)(idx / nrows), i = (int)(idx % nrows);
  float v = 0.f;
  for (int z = 0; z < slices; ++z) v += E[(size_t)z * N * nrows + idx];
  out[(size_t)i * N + n] = v;
}

// max over the sampled rows of |C - ref| / max(1, |ref|) (NaN -> +inf), as int bits in *worst
__global__ void __launch_bounds__(ABFT_THREADS)
rows_max_rel_err(const __bf16* __restrict__ C, const int* __restrict__ rows, int nrows, const float* __restrict__ ref,
                 int N, int* __restrict__ worst) {
  const size_t idx = (size_t)blockIdx.x * ABFT_THREADS + threadIdx.x;
  float rel = 0.f;
  if (idx < (size_t)nrows * N) {
    const int i = (int)(idx / N), n = (int)(idx % N);
    const float got = (float)C[(size_t)rows[i] * N + n], want = ref[idx];
    rel = fabsf(got - want) / fmaxf(1.f, fabsf(want));
    if (!(rel == rel)) rel = __builtin_inff();
  }
  for (int off = 32; off > 0; off >>= 1) rel = fmaxf(rel, __shfl_xor(rel, off));
  if ((threadIdx.x & 63) == 0) atomicMax(worst, __float_as_int(rel));
}

__global__ void abft_inject(__bf16* C, size_t at, float delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) C[at] = (__bf16)((float)C[at] + delta);
}

struct AbftLayout {
  int J, I;          // N-strips (tile columns), M-strips (tile rows)
  ExSplit xr, xc;    // K slicing of the row-check and column-check expectations
  size_t wb, wbabs, wa, waabs, erow, eabsrow, srow, urow, ecol, eabscol, scol, ucol, flags, worst, bytes;
};

AbftLayout abft_layout(int M, int N, int K, int TM, int TN) {
  AbftLayout L{};
  L.J = (N + TN - 1) / TN;
  L.I = (M + TM - 1) / TM;
  L.xr = ex_split(M, L.J, K);
  L.xc = ex_split(N, L.I, K);
  size_t off = 0;
  auto take = [&](size_t floats) {
    const size_t at = off;
    off += (floats * 4 + 255) / 256 * 256;
    return at;
  };
  L.wb = take((size_t)L.J * K);
  L.wbabs = take((size_t)L.J * K);
  L.wa = take((size_t)L.I * K);
  L.waabs = take((size_t)L.I * K);
  L.erow = take((size_t)L.xr.slices * M * L.J);
  L.eabsrow = take((size_t)L.xr.slices * M * L.J);
  L.srow = take((size_t)M * L.J);
  L.urow = take((size_t)M * L.J);
  L.ecol = take((size_t)L.xc.slices * N * L.I);
  L.eabscol = take((size_t)L.xc.slices * N * L.I);
  L.scol = take((size_t)N * L.I);
  L.ucol = take((size_t)N * L.I);
  L.flags = take((size_t)L.I * L.J);
  L.worst = take(1);
  L.bytes = off;
  return L;
}

template <class T>
hipError_t abft_operand_side(const T* A, const T* Bt, int M, int N, int K, int TM, int TN, char* ws,
                             const AbftLayout& L, hipStream_t s) {
  auto at = [&](size_t off) { return (float*)(ws + off); };
  hipLaunchKernelGGL(abft_strip_sums<T>, dim3((K + 255) / 256, L.J), dim3(ABFT_THREADS), 0, s, Bt, N, K, TN,
                     at(L.wb), at(L.wbabs));
  hipLaunchKernelGGL(abft_strip_sums<T>, dim3((K + 255) / 256, L.I), dim3(ABFT_THREADS), 0, s, A, M, K, TM,
                     at(L.wa), at(L.waabs));
  hipLaunchKernelGGL(abft_expect<T>, dim3((M + EX_R - 1) / EX_R, (L.J + EX_J - 1) / EX_J, L.xr.slices),
                     dim3(ABFT_THREADS), 0, s, A, M, K, (const float*)at(L.wb), L.J, L.xr.kper, at(L.erow),
                     at(L.eabsrow));
  hipLaunchKernelGGL(abft_expect<T>, dim3((N + EX_R - 1) / EX_R, (L.I + EX_J - 1) / EX_J, L.xc.slices),
                     dim3(ABFT_THREADS), 0, s, Bt, N, K, (const float*)at(L.wa), L.I, L.xc.kper, at(L.ecol),
                     at(L.eabscol));
  return hipGetLastError();
}

}  // namespace

extern "C" {

// Device workspace the check needs for a shape and tile (bytes).
long long amdgo_abft_workspace_bytes(int M, int N, int K, int TM, int TN) {
  if (M <= 0 || N <= 0 || K <= 0 || TM <= 0 || TN <= 0) return -1;
  return (long long)abft_layout(M, N, K, TM, TN).bytes;
}

// The check of C = A * Bt^T (dtype 0 = bf16, 1 = fp8 e4m3fn operands) in tiles of TM x TN (TN a power
// of two from 64 to 512). On return (the stream synchronised): tile_flags[tm * tiles_n + tn] (host,
// ceil(M/TM) x ceil(N/TN) ints) has bit 0 set when a row sum of that tile failed, bit 1 when a column
// sum did; *worst_ratio (host) is the largest |sum - expected| / tolerance over every sum (< 1 when
// clean). Returns 0, or a hipError_t value.
int amdgo_abft_check(int dtype, const void* A, const void* Bt, const void* C, int M, int N, int K, int TM, int TN,
                     void* ws, long long ws_bytes, int* tile_flags, float* worst_ratio, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || TM <= 0 || (TN != 64 && TN != 128 && TN != 256 && TN != 512) || !ws ||
      !tile_flags || !worst_ratio)
    return (int)hipErrorInvalidValue;
  const AbftLayout L = abft_layout(M, N, K, TM, TN);
  if (ws_bytes < (long long)L.bytes) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  char* w = (char*)ws;
  auto at = [&](size_t off) { return (float*)(w + off); };
  hipError_t e = dtype == 1 ? abft_operand_side((const uint8_t*)A, (const uint8_t*)Bt, M, N, K, TM, TN, w, L, s)
                            : abft_operand_side((const __bf16*)A, (const __bf16*)Bt, M, N, K, TM, TN, w, L, s);
  if (e != hipSuccess) return (int)e;
  const dim3 cg((N + 511) / 512, L.I);
  const __bf16* c = (const __bf16*)C;
  switch (TN) {
    case 64:
      hipLaunchKernelGGL(abft_c_sums<8>, cg, dim3(ABFT_THREADS), 0, s, c, M, N, TM, L.J, L.I, at(L.srow), at(L.urow),
                         at(L.scol), at(L.ucol));
      break;
    case 128:
      hipLaunchKernelGGL(abft_c_sums<16>, cg, dim3(ABFT_THREADS), 0, s, c, M, N, TM, L.J, L.I, at(L.srow), at(L.urow),
                         at(L.scol), at(L.ucol));
      break;
    case 256:
      hipLaunchKernelGGL(abft_c_sums<32>, cg, dim3(ABFT_THREADS), 0, s, c, M, N, TM, L.J, L.I, at(L.srow), at(L.urow),
                         at(L.scol), at(L.ucol));
      break;
    default:
      hipLaunchKernelGGL(abft_c_sums<64>, cg, dim3(ABFT_THREADS), 0, s, c, M, N, TM, L.J, L.I, at(L.srow), at(L.urow),
                         at(L.scol), at(L.ucol));
  }
  int* flags = (int*)(w + L.flags);
  int* worst = (int*)(w + L.worst);
  if ((e = hipMemsetAsync(flags, 0, (size_t)L.I * L.J * 4, s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(worst, 0, 4, s)) != hipSuccess) return (int)e;
  constexpr float kSigma = 4.5f, kRel = 1.0f / 262144.0f;   // see the header
  const size_t nrow = (size_t)M * L.J, ncol = (size_t)N * L.I;
  hipLaunchKernelGGL(abft_compare, dim3((unsigned)((nrow + 255) / 256)), dim3(ABFT_THREADS), 0, s,
                     (const float*)at(L.srow), (const float*)at(L.urow), (const float*)at(L.erow),
                     (const float*)at(L.eabsrow), L.xr.slices, M, L.J, TM, L.J, 0, kSigma, kRel, flags, worst);
  hipLaunchKernelGGL(abft_compare, dim3((unsigned)((ncol + 255) / 256)), dim3(ABFT_THREADS), 0, s,
                     (const float*)at(L.scol), (const float*)at(L.ucol), (const float*)at(L.ecol),
                     (const float*)at(L.eabscol), L.xc.slices, N, L.I, TN, L.J, 1, kSigma, kRel, flags, worst);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if ((e = hipMemcpyAsync(tile_flags, flags, (size_t)L.I * L.J * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return (int)e;
  int wbits = 0;
  if ((e = hipMemcpyAsync(&wbits, worst, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
  std::memcpy(worst_ratio, &wbits, 4);
  return 0;
}

// fp32 reference rows (dtype 0 = bf16, 1 = fp8 e4m3fn operands): out[i][n] = sum_k A[rows[i]][k] Bt[n][k].
// Scratch comes from the stream-ordered pool (hipMallocAsync), released on the stream.
int amdgo_ref_rows(int dtype, const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                   void* stream) {
  if (nrows <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const ExSplit x = ex_split(N, nrows, K);
  float *w = nullptr, *e = nullptr;
  hipError_t err = hipMallocAsync((void**)&w, (size_t)nrows * K * 4, s);
  if (err != hipSuccess) return (int)err;
  if ((err = hipMallocAsync((void**)&e, (size_t)2 * x.slices * N * nrows * 4, s)) != hipSuccess) {
    (void)hipFreeAsync(w, s);
    return (int)err;
  }
  float* eabs = e + (size_t)x.slices * N * nrows;
  const dim3 gg((K + ABFT_THREADS - 1) / ABFT_THREADS < 64 ? (K + ABFT_THREADS - 1) / ABFT_THREADS : 64, nrows);
  const dim3 ge((N + EX_R - 1) / EX_R, (nrows + EX_J - 1) / EX_J, x.slices);
  if (dtype == 1) {
    hipLaunchKernelGGL(gather_rows_f32<uint8_t>, gg, dim3(ABFT_THREADS), 0, s, (const uint8_t*)A, rows, nrows, K, w);
    hipLaunchKernelGGL(abft_expect<uint8_t>, ge, dim3(ABFT_THREADS), 0, s, (const uint8_t*)Bt, N, K, (const float*)w,
                       nrows, x.kper, e, eabs);
  } else {
    hipLaunchKernelGGL(gather_rows_f32<__bf16>, gg, dim3(ABFT_THREADS), 0, s, (const __bf16*)A, rows, nrows, K, w);
    hipLaunchKernelGGL(abft_expect<__bf16>, ge, dim3(ABFT_THREADS), 0, s, (const __bf16*)Bt, N, K, (const float*)w,
                       nrows, x.kper, e, eabs);
  }
  hipLaunchKernelGGL(ref_rows_finish, dim3((unsigned)(((size_t)N * nrows + 255) / 256)), dim3(ABFT_THREADS), 0, s, e,
                     x.slices, N, nrows, out);
  err = hipGetLastError();
  (void)hipFreeAsync(w, s);
  (void)hipFreeAsync(e, s);
  return (int)err;
}

// The sampled-row comparison on the device: *max_rel_err (host; the stream synchronised) = the largest
// |C[rows[i]][n] - ref[i][n]| / max(1, |ref|) over every sampled element (+inf for a NaN). One 4-byte
// readback instead of one copy per row. `scratch`: 4 bytes of device memory.
int amdgo_rows_max_rel_err(const void* C, const int* rows, int nrows, const float* ref, int N, void* scratch,
                           float* max_rel_err, void* stream) {
  if (nrows <= 0 || N <= 0 || !scratch || !max_rel_err) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(scratch, 0, 4, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rows_max_rel_err, dim3((unsigned)(((size_t)nrows * N + 255) / 256)), dim3(ABFT_THREADS), 0, s,
                     (const __bf16*)C, rows, nrows, ref, N, (int*)scratch);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  int bits = 0;
  if ((e = hipMemcpyAsync(&bits, scratch, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
  std::memcpy(max_rel_err, &bits, 4);
  return 0;
}

// Test hook: C[row][col] += delta (one bf16 element; delta NaN makes it NaN), ordered on `stream`.
int amdgo_abft_inject(void* C, int M, int N, int row, int col, float delta, void* stream) {
  if (row < 0 || row >= M || col < 0 || col >= N) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(abft_inject, dim3(1), dim3(64), 0, (hipStream_t)stream, (__bf16*)C, (size_t)row * N + col, delta);
  return (int)hipGetLastError();
}

}  // extern "C"
