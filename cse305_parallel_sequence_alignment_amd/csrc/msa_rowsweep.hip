// msa_rowsweep.hip -- the reference's row sweep in IEEE double, on one CU.
//
// Subproblem::compute_row (alignment_algorithm/subproblem_alignment.cpp:251-327)
// computes row i of T1/T3 elementwise from row i-1 (ComputeRowMapThread13,
// :229-235), then T2 through omega[j] = j*g + max(T1[i][j-1]-g-h, T3[i][j-1]-g-h)
// (ComputeOmegaMapThread :237-242, omega[0] = T2[i][0]), an inclusive prefix
// max (ParallelPrefixMax :13-103) and T2[i][j] = partial[j] - j*g
// (ComputeRowMapThread2 :244-249).  This kernel performs exactly those double
// operations in the same order (no FMA contraction: `fp contract(off)` below,
// so every a*b and a+b rounds on its own as on the reference's x86 build; the
// HIP __d*_rn intrinsics are plain operators that the default contraction mode
// may fuse; max as std::max, (a < b) ? b : a), so every cell is bit-identical to the
// reference for ANY g, h -- the int32 stripe kernels only take integral g, h.
// The prefix max is order-independent, so the block scan below is exact.
//
// One workgroup of 1024 threads sweeps rows [i0, i1) of tables in device
// memory (row stride W = n + 1), or applies one of the reference's per-range
// MapThread bodies to a row (the source-compatible class API).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#pragma clang fp contract(off)

namespace msa {

enum RowPart : int {
  ROW_FIRST = 1,   // ComputeFirstRowMapThread over [start, end) (:212-227)
  ROW_13 = 2,      // ComputeRowMapThread13 over [start, end)
  ROW_OMEGA = 4,   // ComputeOmegaMapThread over [start, end) into vec
  ROW_T2 = 8,      // ComputeRowMapThread2 over [start, end) from vec
  ROW_ZERO = 16,   // compute_row(0) (:259-280)
  ROW_FULL = 32,   // compute_row(i > 0) (:282-326) for i in [i0, i1)
  ROW_SEQ = 64     // with ROW_FULL: T2 by non_parallel_tables' direct recurrence (:398)
};

__device__ __forceinline__ double rmax(double a, double b) { return (a < b) ? b : a; }  // std::max
// one IEEE-rounded operation each (contraction is off in this file)
__device__ __forceinline__ double dmul(double a, double b) { return a * b; }
__device__ __forceinline__ double dadd(double a, double b) { return a + b; }
__device__ __forceinline__ double dsub(double a, double b) { return a - b; }

constexpr int RS_THREADS = 1024;

struct RowArgs {
  double* T1;
  double* T2;
  double* T3;
  long long W;          // row stride (n + 1)
  long long n;
  long long i0, i1;     // absolute rows [i0, i1) (ROW_FULL) or the row (i0) of a part
  long long slot0;      // device row slot of absolute row i0
  const char* A;        // A[k] = the reference's A[id_A + k], k = i0 .. i1-1 (k >= 1)
  const char* B;        // B[j] = the reference's B[id_B + j], j = 1 .. n (B[0] unused)
  double g, h;
  int start_type;
  int part;
  long long start, end;  // column range of a MapThread part
  double* vec;          // omega / partial vector (n + 1) of the OMEGA / T2 parts
};

__device__ __forceinline__ void first_row_cell(const RowArgs& a, double* r1, double* r2, double* r3, long long j) {
  const double NI = -__builtin_inf();
  r1[j] = NI;
  r3[j] = NI;
  if (a.start_type == -2) r2[j] = dmul(-a.g, (double)j);
  else if (a.start_type == 1 || a.start_type == 3) r2[j] = NI;
  else r2[j] = dsub(-a.h, dmul(a.g, (double)j));
}

__device__ __forceinline__ void cell13(const RowArgs& a, const double* u1, const double* u2, const double* u3,
                                       double* r1, double* r3, char ai, long long j) {
  const double f = (ai == a.B[j]) ? 1.0 : 0.0;
  r1[j] = dadd(f, rmax(rmax(u1[j - 1], u2[j - 1]), u3[j - 1]));
  const double gh1 = dsub(dsub(u1[j], a.g), a.h);
  const double gh2 = dsub(dsub(u2[j], a.g), a.h);
  r3[j] = rmax(rmax(gh1, gh2), dsub(u3[j], a.g));
}

__device__ __forceinline__ double omega_of(const RowArgs& a, const double* r1, const double* r3, long long j) {
  const double x = dsub(dsub(r1[j - 1], a.g), a.h);
  const double y = dsub(dsub(r3[j - 1], a.g), a.h);
  return dadd(dmul((double)j, a.g), rmax(x, y));
}

// inclusive prefix max of v[0..n] into out[0..n] (out may alias v)
__device__ void block_prefix_max(const double* v, double* out, long long n, double* lds) {
  const int t = threadIdx.x;
  double carry = -__builtin_inf();
  for (long long base = 0; base <= n; base += RS_THREADS) {
    const long long j = base + t;
    double x = (j <= n) ? v[j] : -__builtin_inf();
    lds[t] = x;
    __syncthreads();
    for (int d = 1; d < RS_THREADS; d <<= 1) {
      const double y = (t >= d) ? lds[t - d] : -__builtin_inf();
      __syncthreads();
      x = rmax(y, x);
      lds[t] = x;
      __syncthreads();
    }
    x = rmax(carry, x);
    if (j <= n) out[j] = x;
    carry = rmax(carry, lds[RS_THREADS - 1]);
    __syncthreads();
  }
}

__global__ __launch_bounds__(RS_THREADS) void rowsweep_kernel(RowArgs a) {
  __shared__ double lds[RS_THREADS];
  const int t = threadIdx.x;
  const long long W = a.W, n = a.n;
  const double NI = -__builtin_inf();
  auto row = [&](double* T, long long i) { return T + (a.slot0 + (i - a.i0)) * W; };
  if (a.part & ROW_ZERO) {
    double *r1 = row(a.T1, a.i0), *r2 = row(a.T2, a.i0), *r3 = row(a.T3, a.i0);
    if (t == 0) {
      r1[0] = NI; r2[0] = NI; r3[0] = NI;
      if (a.start_type == 1 || a.start_type == -1) r1[0] = 0.0;
      else if (a.start_type == -2) r2[0] = 0.0;
      else if (a.start_type == -3) r3[0] = 0.0;
    }
    for (long long j = 1 + t; j <= n; j += RS_THREADS) first_row_cell(a, r1, r2, r3, j);
    return;
  }
  if (a.part & ROW_FIRST) {
    double *r1 = row(a.T1, a.i0), *r2 = row(a.T2, a.i0), *r3 = row(a.T3, a.i0);
    for (long long j = a.start + t; j < a.end; j += RS_THREADS) first_row_cell(a, r1, r2, r3, j);
    return;
  }
  if (a.part & (ROW_13 | ROW_OMEGA | ROW_T2)) {
    const long long i = a.i0;
    double *r1 = row(a.T1, i), *r2 = row(a.T2, i), *r3 = row(a.T3, i);
    if (a.part & ROW_13) {
      const double *u1 = row(a.T1, i - 1), *u2 = row(a.T2, i - 1), *u3 = row(a.T3, i - 1);
      const char ai = a.A[i];
      for (long long j = a.start + t; j < a.end; j += RS_THREADS) cell13(a, u1, u2, u3, r1, r3, ai, j);
    } else if (a.part & ROW_OMEGA) {
      for (long long j = a.start + t; j < a.end; j += RS_THREADS) a.vec[j] = omega_of(a, r1, r3, j);
    } else {
      for (long long j = a.start + t; j < a.end; j += RS_THREADS)
        r2[j] = dsub(a.vec[j], dmul((double)j, a.g));
    }
    return;
  }
  // ROW_FULL: compute_row(i) for every i in [i0, i1), in order
  for (long long i = a.i0; i < a.i1; ++i) {
    double *r1 = row(a.T1, i), *r2 = row(a.T2, i), *r3 = row(a.T3, i);
    const double *u1 = row(a.T1, i - 1), *u2 = row(a.T2, i - 1), *u3 = row(a.T3, i - 1);
    if (t == 0) {  // :282-292
      r1[0] = NI;
      r2[0] = NI;
      if (a.start_type == -3) r3[0] = dmul(-a.g, (double)i);
      else if (a.start_type == 1 || a.start_type == 2) r3[0] = NI;
      else r3[0] = dsub(-a.h, dmul(a.g, (double)i));
    }
    const char ai = a.A[i];
    for (long long j = 1 + t; j <= n; j += RS_THREADS) cell13(a, u1, u2, u3, r1, r3, ai, j);
    __syncthreads();
    if (a.part & ROW_SEQ) {
      // non_parallel_tables (:398): T2[i][j] = max(max(T1[i][j-1]-g-h, T2[i][j-1]-g), T3[i][j-1]-g-h),
      // a serial chain along the row (the reference's sequential twin; differs from the
      // prefix-max form in rounding when g, h are not integral)
      if (t == 0) {
        double prev = r2[0];
        for (long long j = 1; j <= n; ++j) {
          const double x = dsub(dsub(r1[j - 1], a.g), a.h);
          const double y = dsub(prev, a.g);
          const double z = dsub(dsub(r3[j - 1], a.g), a.h);
          prev = rmax(rmax(x, y), z);
          r2[j] = prev;
        }
      }
      __syncthreads();
      continue;
    }
    // omega (:304-312) into the vec scratch, then prefix max in place, then T2
    for (long long j = t; j <= n; j += RS_THREADS) a.vec[j] = (j == 0) ? r2[0] : omega_of(a, r1, r3, j);
    __syncthreads();
    block_prefix_max(a.vec, a.vec, n, lds);
    __syncthreads();
    for (long long j = 1 + t; j <= n; j += RS_THREADS) r2[j] = dsub(a.vec[j], dmul((double)j, a.g));
    __syncthreads();
  }
}

}  // namespace msa
