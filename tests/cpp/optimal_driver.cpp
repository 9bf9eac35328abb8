// optimal_driver.cpp -- TEST DRIVER (tests/test_gpu_refapi.py).
//
// Calls the reference's main_alignment.h API (alignment_algorithm/main_alignment.h:17-38) as a
// reference caller would, linked against libmsa_compat.so.  Built twice: against
// include/main_alignment_compat.h (tests/cpp/Makefile) and, where /root/reference exists, against
// the reference's own unmodified main_alignment.h (oracle/Makefile -> oracle/_ref/optimal_driver_refhdr):
// the second build proves the library is a binary drop-in for that header.
//
// stdin, one case per line (A, B placed 1-based: buffer[0] = '-'):
//   opt g h p m n A B k i0 j0 t0 ... i(k-1) j(k-1) t(k-1)
//       optimal_alignment(A, B, bp, m, n, p, g, h): its stdout is the case's output
//   map g h p start end ida idb m n A B
//       OptimalAlignmentMapThread(...): its bp lines, print_align(begin), "END i j t" (or "END none")
//   sched p m n k i0 j0 t0 ...
//       compute_omega_parallel -> "OMEGA ...", ParallelPrefix -> "SUMS ...", assign_processors per
//       subproblem as optimal_alignment calls it (:244-249) -> "PROCS ...", then the block helpers:
//       ComputeOmegaMapThread over the whole list -> "OMEGA1 ...", PrefixInitMapThread on the
//       whole vector -> "INIT ... | value", PrefixSumMapThread(+7) -> "ADD7 ..."
// Every case ends with "END_CASE"; a thrown exception prints "ERROR <what>" first.
#include <cstdio>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include MAIN_HEADER

static std::vector<align> read_bp(std::istringstream& in) {
  size_t k;
  in >> k;
  std::vector<align> bp(k);
  for (auto& x : bp) {
    in >> x.i >> x.j >> x.t;
    x.next = NULL;
  }
  return bp;
}

static void print_longs(const char* tag, const std::vector<long int>& v) {
  printf("%s", tag);
  for (long int x : v) printf(" %ld", x);
  printf("\n");
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    std::istringstream in(line);
    std::string mode;
    in >> mode;
    try {
      if (mode == "opt") {
        double g, h;
        size_t p, m, n;
        std::string A, B;
        in >> g >> h >> p >> m >> n >> A >> B;
        std::vector<align> bp = read_bp(in);
        std::string a1 = "-" + A, b1 = "-" + B;
        optimal_alignment(&a1[0], &b1[0], bp, m, n, p, g, h);
      } else if (mode == "map") {
        double g, h;
        size_t p, ida, idb, m, n;
        int st, en;
        std::string A, B;
        in >> g >> h >> p >> st >> en >> ida >> idb >> m >> n >> A >> B;
        std::string a1 = "-" + A, b1 = "-" + B;
        align *begin = NULL, *end = NULL;
        OptimalAlignmentMapThread(&a1[0], &b1[0], m, n, ida, idb, p, st, en, g, h, begin, end);
        fflush(stdout);
        print_align(begin);
        if (end) printf("END %zu %zu %d\n", end->i, end->j, end->t);
        else printf("END none\n");
      } else if (mode == "sched") {
        size_t p, m, n;
        in >> p >> m >> n;
        std::vector<align> bp = read_bp(in);
        const size_t num = bp.size() - 1;
        std::vector<long int> omega(num), sums(num);
        compute_omega_parallel(bp, m, n, p, num, omega);
        print_longs("OMEGA", omega);
        ParallelPrefix(p, omega, sums);
        print_longs("SUMS", sums);
        std::vector<long int> procs(num);
        for (size_t i = 0; i < num; ++i)
          procs[i] = (long int)(i == 0 ? assign_processors(0, omega[0]) : assign_processors(sums[i - 1], omega[i]));
        print_longs("PROCS", procs);
        std::vector<long int> omega1(num);
        ComputeOmegaMapThread(bp.begin(), bp.end(), m, n, p, omega1, 0);
        print_longs("OMEGA1", omega1);
        std::vector<long int> init(num);
        queue_indices q;
        q.value = 0;
        q.begin_id = 0;
        q.end_id = num;
        q.next = NULL;
        PrefixInitMapThread(omega, init, q);
        printf("INIT");
        for (long int x : init) printf(" %ld", x);
        printf(" | %ld\n", q.value);
        PrefixSumMapThread(init, 7, &q);
        PrefixSumMapThread(init, 1000, NULL);
        print_longs("ADD7", init);
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
