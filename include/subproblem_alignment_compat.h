/* subproblem_alignment_compat.h -- the reference's `class Subproblem`, source-
 * and binary-compatible, backed by the GPU.
 *
 * Replaces alignment_algorithm/subproblem_alignment.h:8-97 of
 * D-2n/CSE305_Parallel_Sequence_Alignment.  The data members, their order and
 * types, the `align` node and the inline constructor / f / h_prime are those
 * of the reference header (same include guard, so a translation unit sees one
 * of the two), so code written against the reference header -- or compiled
 * with the reference header itself -- links against libmsa_compat.so, which
 * defines the out-of-line members:
 *
 *   compute_tables()      the GPU fill (int32 stripe kernel, msa_subproblem) when g, h are
 *                         integral; otherwise the GPU double row sweep (msa_subproblem_f64),
 *                         bit-identical to subproblem_alignment.cpp:329-355 either way
 *   non_parallel_tables() tables by the direct recurrence (:357-399) on the GPU, printed as :401-421
 *   compute_row(i)        one row of the row sweep on the GPU (:251-327), msa_subproblem_row
 *   ComputeFirstRowMapThread / ComputeRowMapThread13 / ComputeOmegaMapThread /
 *   ComputeRowMapThread2  the per-range bodies (:212-249), on the GPU, msa_subproblem_row
 *   find_alignment()      traceback over this object's T1/T2/T3 (:105-172: tie order, the
 *                         dropped last node Q1, the id_A typo Q2); malloc'd nodes
 *   print_alignment()     :174-180
 *
 * Unlike the reference, a failure (no gfx950 GPU, m = n = 0, a traceback with no
 * matching predecessor) throws std::runtime_error instead of crashing or looping.
 * `p` is kept for signature parity; the GPU path does not depend on it.
 */
#ifndef SUBPROBLEM_ALIGNMENT_H
#define SUBPROBLEM_ALIGNMENT_H

#include <stdio.h>

#include <thread>
#include <vector>

/* a path node (subproblem_alignment.h:8-13) */
typedef struct alignment_point {
  size_t i;
  size_t j;
  int t;
  struct alignment_point* next = NULL;
} align;

class Subproblem {
 public:
  char* A;
  char* B;
  size_t m;     // rows (after the swap: m <= n)
  size_t n;
  size_t id_A;  // offsets into the caller's sequences
  size_t id_B;
  bool invert;  // the constructor swapped A and B (m > n was passed)
  size_t p;     // the reference's processor count (unused by the GPU path)
  int start_type;
  int end_type;
  double g;
  double h;
  std::vector<std::vector<double>> T1;
  std::vector<std::vector<double>> T2;
  std::vector<std::vector<double>> T3;
  align* alignment_begin;
  align* alignment_end;

  /* subproblem_alignment.h:36-74: swap so that m <= n, keep the rest, and size
   * the three (m+1) x (n+1) tables */
  Subproblem(char* _A, char* _B, size_t _m, size_t _n, size_t _id_A, size_t _id_B, size_t _p, int start, int end,
             double _g, double _h) {
    invert = _m > _n;
    A = invert ? _B : _A;
    B = invert ? _A : _B;
    m = invert ? _n : _m;
    n = invert ? _m : _n;
    id_A = invert ? _id_B : _id_A;
    id_B = invert ? _id_A : _id_B;
    p = _p;
    start_type = start;
    end_type = end;
    g = _g;
    h = _h;
    alignment_begin = NULL;
    alignment_end = NULL;
    for (size_t r = 0; r <= m; r++) {
      T1.push_back(std::vector<double>(n + 1));
      T2.push_back(std::vector<double>(n + 1));
      T3.push_back(std::vector<double>(n + 1));
    }
  }

  void non_parallel_tables();
  static void ComputeRowMapThread13(Subproblem* subp, size_t i, size_t start, size_t end);
  static void ComputeOmegaMapThread(Subproblem* subp, size_t i, size_t start, size_t end, std::vector<double>& omega);
  static void ComputeRowMapThread2(Subproblem* subp, size_t i, size_t start, size_t end,
                                   std::vector<double>& partial);
  static void ComputeFirstRowMapThread(Subproblem* subp, size_t start, size_t end);
  void compute_row(size_t i);
  void compute_tables();
  /* substitution (subproblem_alignment.h:83-88): 1 on equal characters, else 0 */
  double f(size_t i, size_t j) { return A[id_A + i] == B[id_B + j] ? 1 : 0; }
  void find_alignment();
  void print_alignment();
  /* subproblem_alignment.h:91-96: h on the end type's own gap table */
  double h_prime(int k) { return (k == end_type && end_type <= -2) ? h : 0; }
};

#endif /* SUBPROBLEM_ALIGNMENT_H */
