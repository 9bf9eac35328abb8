// partial_driver.cpp -- TEST DRIVER (tests/test_gpu_refapi.py).
//
// Calls the reference's partial.h API (sequence_alignment/partial.h:23-41) as a reference caller
// would, linked against libmsa_compat.so.  Built twice: against include/partial_compat.h
// (tests/cpp/Makefile) and, where /root/reference exists, against the reference's own unmodified
// partial.h (oracle/Makefile -> oracle/_ref/partial_driver_refhdr).
//
// stdin, one case per line (A, B 0-based, as partial.cpp reads A[i-1]):
//   part p g h start end A B
//       "PART i j t ..."  findPartialBalancedPartitionParallel(A, B, m, n, p, g, h, start, end, out)
//       "STEP i j t ..."  the same through the step API, as partial.cpp:150-162 composes it:
//                         initializeTables, initializeReverseTables, fillTablesParallel,
//                         fillReverseTablesParallel, findPartitionParallel
//   tabs g h start end A B
//       the six tables after init + fill: "T1" .. "T3" ((m+1) rows), "TR1" .. "TR3" ((m+2) rows)
//   score a b
//       "SCORE s"
// Every case ends with "END_CASE"; a thrown exception prints "ERROR <what>" first.
#include <climits>
#include <cstdio>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include PARTIAL_HEADER

using Table = std::vector<std::vector<int>>;

static void print_points(const char* tag, const std::vector<align>& v) {
  printf("%s", tag);
  for (const align& a : v) printf(" %zu %zu %d", a.i, a.j, a.t);
  printf("\n");
}

static void fill_all(const std::string& A, const std::string& B, double g, double h, int st, int en, Table* T,
                     Table* R) {
  const size_t m = A.size(), n = B.size();
  for (int v = 0; v < 3; ++v) {
    T[v].assign(m + 1, std::vector<int>(n + 1));
    R[v].assign(m + 2, std::vector<int>(n + 2, INT_MIN));
  }
  initializeTables(T[0], T[1], T[2], m, n, g, h, st);
  initializeReverseTables(R[0], R[1], R[2], m, n, g, h, en);
  fillTablesParallel(A.data(), B.data(), m, n, T[0], T[1], T[2], g, h, 4);
  fillReverseTablesParallel(A.data(), B.data(), m, n, R[0], R[1], R[2], g, h, 4);
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    std::istringstream in(line);
    std::string mode;
    in >> mode;
    try {
      if (mode == "part") {
        size_t p;
        double g, h;
        int st, en;
        std::string A, B;
        in >> p >> g >> h >> st >> en >> A >> B;
        std::vector<align> out;
        findPartialBalancedPartitionParallel(A.data(), B.data(), A.size(), B.size(), p, g, h, st, en, out);
        print_points("PART", out);
        Table T[3], R[3];
        fill_all(A, B, g, h, st, en, T, R);
        print_points("STEP", findPartitionParallel(T[0], T[1], T[2], R[0], R[1], R[2], A.size(), B.size(), p, h));
      } else if (mode == "tabs") {
        double g, h;
        int st, en;
        std::string A, B;
        in >> g >> h >> st >> en >> A >> B;
        Table T[3], R[3];
        fill_all(A, B, g, h, st, en, T, R);
        const char* names[6] = {"T1", "T2", "T3", "TR1", "TR2", "TR3"};
        for (int v = 0; v < 6; ++v) {
          printf("%s\n", names[v]);
          for (const auto& row : (v < 3 ? T[v] : R[v - 3])) {
            for (int x : row) printf("%d ", x);
            printf("\n");
          }
        }
      } else if (mode == "score") {
        std::string a, b;
        in >> a >> b;
        printf("SCORE %d\n", score(a[0], b[0]));
      }
    } catch (const std::exception& e) {
      fflush(stdout);
      printf("ERROR %s\n", e.what());
    }
    printf("END_CASE\n");
    fflush(stdout);
  }
  return 0;
}
