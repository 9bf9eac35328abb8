// subproblem_compat.cpp -- out-of-line members of the reference's `class
// Subproblem` (include/subproblem_alignment_compat.h), over the C-ABI of
// libmsa.so.  Every table cell is computed on the GPU; this file moves rows
// between the caller's vector<vector<double>> tables and the C-ABI, and walks
// the traceback over those tables the way subproblem_alignment.cpp:105-172 does.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "msa.h"
#include "subproblem_alignment_compat.h"

namespace {

void check(int rc, const char* what) {
  if (rc != MSA_OK)
    throw std::runtime_error(std::string("Subproblem::") + what + ": " + msa_status_string(rc) + " (status " +
                             std::to_string(rc) + ")");
}

// flat (m+1) x (n+1) row-major doubles -> the object's tables
void store(Subproblem* s, const std::vector<double>* flat) {
  std::vector<std::vector<double>>* T[3] = {&s->T1, &s->T2, &s->T3};
  const size_t W = s->n + 1;
  for (int v = 0; v < 3; ++v) {
    T[v]->resize(s->m + 1);
    for (size_t i = 0; i <= s->m; ++i) (*T[v])[i].assign(flat[v].begin() + i * W, flat[v].begin() + (i + 1) * W);
  }
}

// the object's tables, filled by the GPU: `mode` = MSA_F64_COMPUTE_TABLES (compute_tables'
// prefix-max T2) or MSA_F64_NON_PARALLEL (non_parallel_tables' direct recurrence)
void fill(Subproblem* s, int mode, const char* what) {
  const size_t cells = (s->m + 1) * (s->n + 1);
  std::vector<double> flat[3];
  for (auto& f : flat) f.resize(cells);
  // integral g, h: the int32 stripe kernel (bit-identical to both forms); INT32_MIN = -inf
  std::vector<int32_t> ti[3];
  for (auto& t : ti) t.resize(cells);
  const int rc = msa_subproblem(s->A, s->B, s->m, s->n, s->id_A, s->id_B, s->start_type, s->end_type, s->g, s->h,
                                ti[0].data(), ti[1].data(), ti[2].data(), nullptr, 0, nullptr, nullptr, nullptr);
  if (rc == MSA_OK) {
    for (int v = 0; v < 3; ++v)
      for (size_t e = 0; e < cells; ++e) flat[v][e] = ti[v][e] == INT32_MIN ? -INFINITY : (double)ti[v][e];
  } else if (rc == MSA_ERR_UNSUPPORTED) {  // any other g, h: the double row sweep
    check(msa_subproblem_f64(s->A, s->B, s->m, s->n, s->id_A, s->id_B, s->start_type, s->g, s->h, mode,
                             flat[0].data(), flat[1].data(), flat[2].data(), nullptr),
          what);
  } else {
    check(rc, what);
  }
  store(s, flat);
}

void row_part(int part, Subproblem* s, size_t i, size_t start, size_t end, double* vec, const char* what) {
  const double* up[3] = {nullptr, nullptr, nullptr};
  if (part == MSA_ROW_13 || part == MSA_ROW_FULL) {
    up[0] = s->T1[i - 1].data();
    up[1] = s->T2[i - 1].data();
    up[2] = s->T3[i - 1].data();
  }
  check(msa_subproblem_row(part, s->A, s->B, s->id_A, s->id_B, s->n, i, s->start_type, s->g, s->h, start, end,
                           up[0], up[1], up[2], s->T1[i].data(), s->T2[i].data(), s->T3[i].data(), vec),
        what);
}

}  // namespace

void Subproblem::compute_tables() { fill(this, MSA_F64_COMPUTE_TABLES, "compute_tables"); }

void Subproblem::non_parallel_tables() {
  fill(this, MSA_F64_NON_PARALLEL, "non_parallel_tables");
  // subproblem_alignment.cpp:401-421
  const std::vector<std::vector<double>>* T[3] = {&T1, &T2, &T3};
  for (int v = 0; v < 3; ++v) {
    printf("T%d:\n", v + 1);
    for (size_t i = 0; i <= m; i++) {
      for (size_t j = 0; j <= n; j++) printf("%lf ", (*T[v])[i][j]);
      printf("\n");
    }
  }
}

void Subproblem::compute_row(size_t i) {
  row_part(i == 0 ? MSA_ROW_ZERO : MSA_ROW_FULL, this, i, 0, 0, nullptr, "compute_row");
}

void Subproblem::ComputeFirstRowMapThread(Subproblem* subp, size_t start, size_t end) {
  row_part(MSA_ROW_FIRST, subp, 0, start, end, nullptr, "ComputeFirstRowMapThread");
}

void Subproblem::ComputeRowMapThread13(Subproblem* subp, size_t i, size_t start, size_t end) {
  row_part(MSA_ROW_13, subp, i, start, end, nullptr, "ComputeRowMapThread13");
}

void Subproblem::ComputeOmegaMapThread(Subproblem* subp, size_t i, size_t start, size_t end,
                                       std::vector<double>& omega) {
  omega.resize(subp->n + 1);
  row_part(MSA_ROW_OMEGA, subp, i, start, end, omega.data(), "ComputeOmegaMapThread");
}

void Subproblem::ComputeRowMapThread2(Subproblem* subp, size_t i, size_t start, size_t end,
                                      std::vector<double>& partial) {
  partial.resize(subp->n + 1);
  row_part(MSA_ROW_T2, subp, i, start, end, partial.data(), "ComputeRowMapThread2");
}

// subproblem_alignment.cpp:105-172 over this object's tables (exact double
// equality, first of T1, T2, T3); the list runs alignment_begin -> alignment_end
void Subproblem::find_alignment() {
  size_t i = m, j = n;
  align* cur = (align*)std::malloc(sizeof(align));
  if (!cur) throw std::bad_alloc();
  cur->next = NULL;
  alignment_end = cur;
  if (end_type > 0) {
    cur->t = end_type;
    cur->i = (end_type == 2) ? 0 : i + id_A;
    cur->j = (end_type == 3) ? 0 : j + id_B;
  } else {
    const double t1 = T1[m][n], t2 = T2[m][n] + h_prime(-2), t3 = T3[m][n] + h_prime(-3);
    if (t1 >= t2 && t1 >= t3) {
      cur->t = 1; cur->i = i + id_A; cur->j = j + id_B;
    } else if (t2 >= t1 && t2 >= t3) {
      cur->t = 2; cur->i = 0; cur->j = j + id_B;
    } else {
      cur->t = 3; cur->i = i + id_A; cur->j = 0;
    }
  }
  while (i > 0 && j > 0) {
    align* nw = (align*)std::malloc(sizeof(align));
    if (!nw) throw std::bad_alloc();
    int nt = 0;
    if (cur->t == 1) {
      const double v = T1[i][j], fij = f(i, j);
      if (v == fij + T1[i - 1][j - 1]) { nt = 1; nw->i = i - 1 + id_A; nw->j = j - 1 + id_A; }  // Q2 (:151)
      else if (v == fij + T2[i - 1][j - 1]) { nt = 2; nw->i = 0; nw->j = j - 1 + id_B; }
      else if (v == fij + T3[i - 1][j - 1]) { nt = 3; nw->i = i - 1 + id_A; nw->j = 0; }
      if (nt) { i--; j--; }
    } else if (cur->t == 2) {
      const double v = T2[i][j];
      if (v == -g - h + T1[i][j - 1]) { nt = 1; nw->i = i + id_A; nw->j = j - 1 + id_B; }
      else if (v == -g + T2[i][j - 1]) { nt = 2; nw->i = 0; nw->j = j - 1 + id_B; }
      else if (v == -g - h + T3[i][j - 1]) { nt = 3; nw->i = i + id_A; nw->j = 0; }
      if (nt) j--;
    } else {
      const double v = T3[i][j];
      if (v == -g - h + T1[i - 1][j]) { nt = 1; nw->i = i - 1 + id_A; nw->j = j + id_B; }
      else if (v == -g - h + T2[i - 1][j]) { nt = 2; nw->i = 0; nw->j = j + id_B; }
      else if (v == -g + T3[i - 1][j]) { nt = 3; nw->i = i - 1 + id_A; nw->j = 0; }
      if (nt) i--;
    }
    if (!nt) {  // the reference loops forever here (uninitialised node, :147-169)
      std::free(nw);
      throw std::runtime_error("Subproblem::find_alignment: no predecessor matches the tables");
    }
    nw->t = nt;
    nw->next = cur;
    cur = nw;
  }
  alignment_begin = cur->next;  // Q1: the last-created node is not part of the list (:170)
}

void Subproblem::print_alignment() {
  for (align* a = alignment_begin; a != NULL; a = a->next) printf("(%ld, %ld, %d)\n", a->i, a->j, a->t);
}
