// ref_partial_driver.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// extern "C" driver around the reference's unmodified
// sequence_alignment/partial.{h,cpp}, compiled straight from /root/reference
// at -O0 like the reference Makefile (Makefile:3), whose int32 overflow at the
// INT_MIN sentinels then wraps.  Fixture generator input only.
#include <cstring>
#include <vector>

#include "partial.h"

extern "C" {

int ref_partial(const char* A, const char* B, size_t m, size_t n, size_t p, double g, double h, int start_type,
                int end_type, size_t cap, size_t* n_out, unsigned long long* oi, unsigned long long* oj, int* ot) {
  std::vector<align> part;
  findPartialBalancedPartitionParallel(A, B, m, n, p, g, h, start_type, end_type, part);
  *n_out = part.size();
  for (size_t k = 0; k < part.size() && k < cap; k++) {
    oi[k] = part[k].i;
    oj[k] = part[k].j;
    ot[k] = part[k].t;
  }
  return 0;
}

// The six tables findPartialBalancedPartitionParallel builds (partial.cpp:150-161).
int ref_partial_tables(const char* A, const char* B, size_t m, size_t n, size_t p, double g, double h,
                       int start_type, int end_type, int* T1o, int* T2o, int* T3o, int* R1o, int* R2o, int* R3o) {
  std::vector<std::vector<int>> T1(m + 1, std::vector<int>(n + 1));
  std::vector<std::vector<int>> T2(m + 1, std::vector<int>(n + 1));
  std::vector<std::vector<int>> T3(m + 1, std::vector<int>(n + 1));
  std::vector<std::vector<int>> TR1(m + 2, std::vector<int>(n + 2, INT_MIN));
  std::vector<std::vector<int>> TR2(m + 2, std::vector<int>(n + 2, INT_MIN));
  std::vector<std::vector<int>> TR3(m + 2, std::vector<int>(n + 2, INT_MIN));
  initializeTables(T1, T2, T3, m, n, g, h, start_type);
  initializeReverseTables(TR1, TR2, TR3, m, n, g, h, end_type);
  fillTablesParallel(A, B, m, n, T1, T2, T3, g, h, p);
  fillReverseTablesParallel(A, B, m, n, TR1, TR2, TR3, g, h, p);
  for (size_t i = 0; i <= m; i++) {
    std::memcpy(T1o + i * (n + 1), T1[i].data(), sizeof(int) * (n + 1));
    std::memcpy(T2o + i * (n + 1), T2[i].data(), sizeof(int) * (n + 1));
    std::memcpy(T3o + i * (n + 1), T3[i].data(), sizeof(int) * (n + 1));
  }
  for (size_t i = 0; i <= m + 1; i++) {
    std::memcpy(R1o + i * (n + 2), TR1[i].data(), sizeof(int) * (n + 2));
    std::memcpy(R2o + i * (n + 2), TR2[i].data(), sizeof(int) * (n + 2));
    std::memcpy(R3o + i * (n + 2), TR3[i].data(), sizeof(int) * (n + 2));
  }
  return 0;
}

}  // extern "C"
