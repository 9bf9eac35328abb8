// partial_compat.cpp -- the reference's sequence_alignment/partial.h API with its C++ signatures
// (include/partial_compat.h), over the C-ABI of libmsa.so.  Own translation unit: partial.h's `align`
// and subproblem_alignment.h's are two definitions of one name.  The forward / reverse fills and the
// partition's band maxima run on the GPU (msa_partial_tables, msa_partition_tables,
// msa_partial_partition); this file moves the caller's vector<vector<int>> tables across the C-ABI
// and writes initializeTables' borders (no DP cell).
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "msa.h"
#include "partial_compat.h"

namespace {

using Table = std::vector<std::vector<int>>;

[[noreturn]] void fail(const char* fn, int rc) {
  const std::string msg = std::string(fn) + ": " + msa_status_string(rc) + " (status " + std::to_string(rc) + ")";
  if (rc == MSA_ERR_ARG) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

// partial.cpp's gap cells -(int)(g + h) * k: an int times a size_t, kept as an int (mod 2^32)
int gap_cell(int GH, size_t k) { return (int)(uint32_t)((size_t)(-(long long)GH) * k); }

// The border cells initializeTables (partial.cpp:13-31) gives start type st, compared with the
// caller's row 0 and column 0 (the only cells fillTablesParallel reads and does not write).
bool forward_borders(const Table& T1, const Table& T2, const Table& T3, size_t m, size_t n, int GH, int st) {
  for (size_t j = 0; j <= n; ++j) {
    const int t1 = (j == 0 && st == 1) ? 0 : INT_MIN;
    const int t2 = (j >= 1 && st == 2) ? gap_cell(GH, j) : INT_MIN;
    if (T1[0][j] != t1 || T2[0][j] != t2 || T3[0][j] != INT_MIN) return false;
  }
  for (size_t i = 1; i <= m; ++i) {
    const int t3 = (st == 3) ? gap_cell(GH, i) : INT_MIN;
    if (T1[i][0] != INT_MIN || T2[i][0] != INT_MIN || T3[i][0] != t3) return false;
  }
  return true;
}

// initializeReverseTables (partial.cpp:33-51): row m+1 and column n+1, the cells the reverse fill reads
bool reverse_borders(const Table& R1, const Table& R2, const Table& R3, size_t m, size_t n, int GH, int et) {
  for (size_t j = 0; j <= n + 1; ++j) {
    const int r1 = (j == n + 1 && et == 1) ? 0 : INT_MIN;
    const int r2 = (j >= 1 && j <= n && et == 2) ? gap_cell(GH, n - j + 1) : INT_MIN;
    if (R1[m + 1][j] != r1 || R2[m + 1][j] != r2 || R3[m + 1][j] != INT_MIN) return false;
  }
  for (size_t i = 0; i <= m; ++i) {
    const int r3 = (i >= 1 && et == 3) ? gap_cell(GH, m - i + 1) : INT_MIN;
    if (R1[i][n + 1] != INT_MIN || R2[i][n + 1] != INT_MIN || R3[i][n + 1] != r3) return false;
  }
  return true;
}

void check_shape(const Table& T, size_t rows, size_t cols, const char* fn) {
  if (T.size() < rows) throw std::invalid_argument(std::string(fn) + ": table has fewer rows than the fill reads");
  for (size_t i = 0; i < rows; ++i)
    if (T[i].size() < cols) throw std::invalid_argument(std::string(fn) + ": table row shorter than the fill reads");
}

std::vector<int32_t> flat(const Table& T, size_t rows, size_t cols) {
  std::vector<int32_t> f(rows * cols);
  for (size_t i = 0; i < rows; ++i) std::memcpy(f.data() + i * cols, T[i].data(), cols * sizeof(int32_t));
  return f;
}

}  // namespace

// partial.cpp:9-11 (match 0, mismatch 1: the reference's scoring under max)
int score(char a, char b) { return (a == b) ? 0 : 1; }

void initializeTables(Table& T1, Table& T2, Table& T3, size_t m, size_t n, double g, double h, int start_type) {
  const int GH = (int)(g + h);
  for (size_t i = 0; i <= m; ++i)
    for (size_t j = 0; j <= n; ++j) T1[i][j] = T2[i][j] = T3[i][j] = INT_MIN;
  if (start_type == 1) {
    T1[0][0] = 0;
  } else if (start_type == 2) {
    for (size_t j = 1; j <= n; ++j) T2[0][j] = gap_cell(GH, j);
  } else if (start_type == 3) {
    for (size_t i = 1; i <= m; ++i) T3[i][0] = gap_cell(GH, i);
  }
}

void initializeReverseTables(Table& TR1, Table& TR2, Table& TR3, size_t m, size_t n, double g, double h,
                             int end_type) {
  const int GH = (int)(g + h);
  for (size_t i = 0; i <= m + 1; ++i)
    for (size_t j = 0; j <= n + 1; ++j) TR1[i][j] = TR2[i][j] = TR3[i][j] = INT_MIN;
  if (end_type == 1) {
    TR1[m + 1][n + 1] = 0;
  } else if (end_type == 2) {
    for (size_t j = 1; j <= n; ++j) TR2[m + 1][j] = gap_cell(GH, n - j + 1);
  } else if (end_type == 3) {
    for (size_t i = 1; i <= m; ++i) TR3[i][n + 1] = gap_cell(GH, m - i + 1);
  }
}

// partial.cpp:53-65: cells (1..m) x (1..n) of the forward tables from the GPU
void fillTablesParallel(const char* A, const char* B, size_t m, size_t n, Table& T1, Table& T2, Table& T3, double g,
                        double h, size_t p) {
  (void)p;  // the reference's (inert) OpenMP thread count
  if (m == 0 || n == 0) return;
  for (const Table* T : {&T1, &T2, &T3}) check_shape(*T, m + 1, n + 1, "fillTablesParallel");
  const int GH = (int)(g + h);
  int st = -1;
  for (int c : {1, 2, 3, 0})
    if (forward_borders(T1, T2, T3, m, n, GH, c)) {
      st = c;
      break;
    }
  if (st < 0)
    throw std::invalid_argument("fillTablesParallel: the tables' borders are not those initializeTables writes");
  std::vector<int32_t> out[3];
  for (auto& o : out) o.resize((m + 1) * (n + 1));
  const int rc = msa_partial_tables(A, B, m, n, g, h, st, 0, out[0].data(), out[1].data(), out[2].data(), nullptr,
                                    nullptr, nullptr);
  if (rc != MSA_OK) fail("fillTablesParallel", rc);
  Table* T[3] = {&T1, &T2, &T3};
  for (int v = 0; v < 3; ++v)
    for (size_t i = 1; i <= m; ++i)
      std::memcpy((*T[v])[i].data() + 1, out[v].data() + i * (n + 1) + 1, n * sizeof(int32_t));
}

// partial.cpp:67-79: cells (1..m) x (1..n) of the reverse tables from the GPU
void fillReverseTablesParallel(const char* A, const char* B, size_t m, size_t n, Table& TR1, Table& TR2, Table& TR3,
                               double g, double h, size_t p) {
  (void)p;
  if (m == 0 || n == 0) return;
  for (const Table* T : {&TR1, &TR2, &TR3}) check_shape(*T, m + 2, n + 2, "fillReverseTablesParallel");
  const int GH = (int)(g + h);
  int et = -1;
  for (int c : {1, 2, 3, 0})
    if (reverse_borders(TR1, TR2, TR3, m, n, GH, c)) {
      et = c;
      break;
    }
  if (et < 0)
    throw std::invalid_argument(
        "fillReverseTablesParallel: the tables' borders are not those initializeReverseTables writes");
  std::vector<int32_t> out[3];
  for (auto& o : out) o.resize((m + 2) * (n + 2));
  const int rc = msa_partial_tables(A, B, m, n, g, h, 0, et, nullptr, nullptr, nullptr, out[0].data(), out[1].data(),
                                    out[2].data());
  if (rc != MSA_OK) fail("fillReverseTablesParallel", rc);
  Table* T[3] = {&TR1, &TR2, &TR3};
  for (int v = 0; v < 3; ++v)
    for (size_t i = 1; i <= m; ++i)
      std::memcpy((*T[v])[i].data() + 1, out[v].data() + i * (n + 2) + 1, n * sizeof(int32_t));
}

// partial.cpp:81-146 over the caller's tables (band maxima on the GPU)
std::vector<align> findPartitionParallel(const Table& T1, const Table& T2, const Table& T3, const Table& TR1,
                                         const Table& TR2, const Table& TR3, size_t m, size_t n, size_t p, double h) {
  if (p == 0) throw std::invalid_argument("findPartitionParallel: p = 0 (the reference divides by it)");
  for (const Table* T : {&T1, &T2, &T3}) check_shape(*T, m + 1, n + 1, "findPartitionParallel");
  for (const Table* T : {&TR1, &TR2, &TR3}) check_shape(*T, m + 2, n + 2, "findPartitionParallel");
  const std::vector<int32_t> f1 = flat(T1, m + 1, n + 1), f2 = flat(T2, m + 1, n + 1), f3 = flat(T3, m + 1, n + 1);
  const std::vector<int32_t> r1 = flat(TR1, m + 2, n + 2), r2 = flat(TR2, m + 2, n + 2), r3 = flat(TR3, m + 2, n + 2);
  std::vector<msa_node> pts(p + 1);
  size_t np = 0;
  const int rc = msa_partition_tables(f1.data(), f2.data(), f3.data(), r1.data(), r2.data(), r3.data(), m, n, p, h,
                                      pts.data(), pts.size(), &np);
  if (rc != MSA_OK) fail("findPartitionParallel", rc);
  std::vector<align> out;
  out.reserve(np);
  for (size_t k = 0; k < np; ++k) out.push_back({(size_t)pts[k].i, (size_t)pts[k].j, pts[k].t, nullptr});
  return out;
}

// partial.cpp:149-163: forward + reverse fills and the partition, all on the GPU
void findPartialBalancedPartitionParallel(const char* A, const char* B, size_t m, size_t n, size_t p, double g,
                                          double h, int start_type, int end_type, std::vector<align>& partition) {
  std::vector<msa_node> pts(p + 1);
  size_t np = 0;
  const int rc =
      msa_partial_partition(A, B, m, n, p, g, h, start_type, end_type, pts.data(), pts.size(), &np);
  if (rc != MSA_OK) fail("findPartialBalancedPartitionParallel", rc);
  partition.clear();
  for (size_t k = 0; k < np; ++k) partition.push_back({(size_t)pts[k].i, (size_t)pts[k].j, pts[k].t, nullptr});
}
