// subproblem_driver.cpp -- TEST DRIVER (tests/test_gpu_refapi.py).
//
// Exercises the reference's `class Subproblem` API exactly as a reference
// caller would (subproblem_alignment.h:16-97), linked against libmsa_compat.so.
// Built twice: against include/subproblem_alignment_compat.h (tests/cpp/Makefile)
// and, where /root/reference exists, against the reference's own unmodified
// subproblem_alignment.h (oracle/Makefile -> oracle/_ref/subproblem_driver_refhdr):
// the second build proves the library is a binary drop-in for the reference header.
//
// stdin, one case per line:   mode g h start end p idA idB m n A B
//   mode tables : ctor, compute_tables(), find_alignment()
//   mode rows   : ctor, compute_row(i) for i = 0..m  (subproblem_alignment.cpp:329-332)
//   mode maps   : ctor, then each row as compute_row does it (:251-327) but through the
//                 static MapThread bodies, three column ranges on three std::threads
//   mode nonpar : ctor, non_parallel_tables() (prints the tables itself)
// A and B are the sequences (placed 1-based: buffer[0] = '-').
// stdout: "INV x", the three tables as C99 hex floats ("%a"), "NODES k" + k lines
// "i j t", "END i j t" (mode tables), then "END_CASE".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include SUBPROBLEM_HEADER

static void print_tables(Subproblem& s) {
  std::vector<std::vector<double>>* T[3] = {&s.T1, &s.T2, &s.T3};
  for (int v = 0; v < 3; ++v) {
    printf("T%d\n", v + 1);
    for (size_t i = 0; i <= s.m; ++i) {
      for (size_t j = 0; j <= s.n; ++j) printf("%a ", (*T[v])[i][j]);
      printf("\n");
    }
  }
}

// compute_row(i > 0) restated over the static bodies; the borders and the prefix
// max are the driver's (test-side) part, the cells come from the library
static void row_by_maps(Subproblem& s, size_t i) {
  const double NI = -INFINITY;
  s.T1[i][0] = NI;
  s.T2[i][0] = NI;
  if (s.start_type == -3) s.T3[i][0] = -s.g * i;
  else if (s.start_type == 1 || s.start_type == 2) s.T3[i][0] = NI;
  else s.T3[i][0] = -s.h - s.g * i;
  const size_t n = s.n, k = std::min<size_t>(3, n), bs = n / k;
  auto ranges = [&](auto fn) {
    std::vector<std::thread> th;
    for (size_t t = 0; t < k; ++t) {
      const size_t a = 1 + t * bs, b = (t + 1 == k) ? n + 1 : 1 + (t + 1) * bs;
      th.emplace_back(fn, a, b);
    }
    for (auto& x : th) x.join();
  };
  ranges([&](size_t a, size_t b) { Subproblem::ComputeRowMapThread13(&s, i, a, b); });
  std::vector<double> omega(n + 1), partial(n + 1);
  omega[0] = s.T2[i][0];
  ranges([&](size_t a, size_t b) { Subproblem::ComputeOmegaMapThread(&s, i, a, b, omega); });
  double run = omega[0];
  for (size_t j = 0; j <= n; ++j) partial[j] = run = std::max(run, omega[j]);
  ranges([&](size_t a, size_t b) { Subproblem::ComputeRowMapThread2(&s, i, a, b, partial); });
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    std::istringstream in(line);
    std::string mode, A, B;
    double g, h;
    int st, en;
    size_t p, idA, idB, m, n;
    in >> mode >> g >> h >> st >> en >> p >> idA >> idB >> m >> n >> A >> B;
    std::string a1 = "-" + A, b1 = "-" + B;
    try {
      Subproblem s(&a1[0], &b1[0], m, n, idA, idB, p, st, en, g, h);
      printf("INV %d\n", s.invert ? 1 : 0);
      if (mode == "tables") {
        s.compute_tables();
      } else if (mode == "rows") {
        for (size_t i = 0; i <= s.m; ++i) s.compute_row(i);
      } else if (mode == "maps") {
        s.compute_row(0);
        for (size_t i = 1; i <= s.m; ++i) row_by_maps(s, i);
      } else if (mode == "nonpar") {
        s.non_parallel_tables();
        printf("END_CASE\n");
        continue;
      }
      print_tables(s);
      if (mode == "tables") {
        s.find_alignment();
        size_t k = 0;
        for (align* x = s.alignment_begin; x; x = x->next) ++k;
        printf("NODES %zu\n", k);
        for (align* x = s.alignment_begin; x; x = x->next) printf("%zu %zu %d\n", x->i, x->j, x->t);
        printf("END %zu %zu %d\n", s.alignment_end->i, s.alignment_end->j, s.alignment_end->t);
      }
    } catch (const std::exception& e) {
      printf("ERROR %s\n", e.what());
    }
    printf("END_CASE\n");
    fflush(stdout);
  }
  return 0;
}
