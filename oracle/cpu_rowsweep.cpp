// cpu_rowsweep.cpp -- TEST INFRASTRUCTURE ONLY: the CPU baseline.
//
// The build's own restatement of the reference's CPU algorithm, so that
// bench.py's `cpu_baseline` times the reference's *method* on the GPU box's
// host cores without shipping reference sources or binaries there (SURVEY.md
// §8(c)/(d)(ii)).  Nothing in the product links or loads this file.
//
// The method (alignment_algorithm/subproblem_alignment.cpp):
//   * Subproblem::compute_tables (:329-332) sweeps rows i = 0..m;
//   * compute_row(i) (:251-327) splits the columns into p' blocks (:252-257)
//     and, per row, runs FRESH std::threads for each phase:
//       1. ComputeRowMapThread13 (:229-235)  -- cells that depend on row i-1 only,
//       2. ComputeOmegaMapThread (:237-242)  -- omega[j] = j*g + (left-open candidate),
//       3. ParallelPrefixMax (:13-103)       -- per-block prefix max, then
//          pointer-jumping rounds that max each block with its predecessor's value,
//       4. ComputeRowMapThread2 (:244-249)   -- T2[i][j] = prefmax[j] - j*g;
//   * main_alignment_function maps the harness's p to p' = (p+2)/3
//     (main_alignment.cpp:192-200), so p = 32 runs p' = 11.
//
// Two recurrences run through that same method:
//   mode 0  the reference's own global Gotoh in double with -inf
//           (T1/T2/T3, start type -1, f = 1 if equal else 0, open g+h, extend g);
//           score = max(T1,T2,T3)[m][n]  (equals orc_subproblem_tables);
//   mode 1  BASELINE config C2/C4's Smith-Waterman with linear gap in int32:
//           Tv(i,j) = max(0, H(i-1,j-1) + s, H(i-1,j) - g)      (phase 1)
//           omega[j] = Tv(i,j) + j*g, omega[0] = H(i,0) = 0      (phase 2)
//           H(i,j) = prefmax(omega)[j] - j*g                     (phases 3-4)
//           i.e. the reference's T2 prefix-max trick applied to the horizontal
//           gap; score = max H (equals orc_sw's score).
// Two rows are kept (the reference keeps all m+1; the fill arithmetic and the
// thread structure are the same).  `rows` bounds the sample: rows 1..rows are
// filled and timed (GCUPS = rows * n / seconds).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <thread>
#include <utility>
#include <vector>

namespace {

// Run f(start, end) over p' column blocks of [1, n], blocks 0..p'-2 on fresh
// threads and the last on the caller (compute_row's pattern, :295-301).
template <class F>
void map_blocks(size_t n, size_t p, F&& f) {
  size_t block = n / p, nt = p;
  if (p > n) {
    nt = n;
    block = 1;
  }
  std::vector<std::thread> workers;
  workers.reserve(nt - 1);
  for (size_t j = 0; j + 1 < nt; ++j) workers.emplace_back(f, 1 + j * block, 1 + (j + 1) * block);
  f(1 + (nt - 1) * block, n + 1);
  for (auto& w : workers) w.join();
}

// ParallelPrefixMax (:13-103): values[0..N) -> out[0..N), p blocks, fresh threads.
template <class T>
void prefix_max(size_t p, const std::vector<T>& values, std::vector<T>& out) {
  const size_t N = values.size();
  size_t block = N / p, parts = p;
  if (p > N) {
    block = 1;
    parts = N;
  }
  struct Unit {
    size_t b, e;
    long next;
  };
  std::vector<Unit> u(parts);
  for (size_t i = 0; i < parts; ++i) {
    u[i].b = block * i;
    u[i].e = (i == parts - 1 || block * (i + 1) >= N) ? N : block * (i + 1);
    u[i].next = (i + 1 < parts) ? (long)(i + 1) : -1;
  }
  auto init = [&](size_t k) {
    out[u[k].b] = values[u[k].b];
    for (size_t i = u[k].b + 1; i < u[k].e; ++i) out[i] = std::max(out[i - 1], values[i]);
  };
  {
    std::vector<std::thread> w;
    for (size_t k = 1; k < parts; ++k) w.emplace_back(init, k);
    init(0);
    for (auto& t : w) t.join();
  }
  // pointer jumping: every live unit q with a successor r maxes r's block with
  // q's last prefix value, then links past r (the reference's deque rounds)
  std::vector<size_t> live(parts);
  for (size_t k = 0; k < parts; ++k) live[k] = k;
  while (!live.empty()) {
    std::vector<size_t> nxt;
    std::vector<std::pair<T, long>> jobs;
    for (size_t q : live) {
      if (u[q].next < 0) continue;
      const long r = u[q].next;
      jobs.emplace_back(out[u[q].e - 1], r);
      u[q].next = u[(size_t)r].next;
      nxt.push_back(q);
    }
    auto apply = [&](size_t k) {
      const T v = jobs[k].first;
      const Unit& r = u[(size_t)jobs[k].second];
      for (size_t i = r.b; i < r.e; ++i) out[i] = std::max(out[i], v);
    };
    std::vector<std::thread> w;
    for (size_t k = 1; k < jobs.size(); ++k) w.emplace_back(apply, k);
    if (!jobs.empty()) apply(0);
    for (auto& t : w) t.join();
    live.swap(nxt);
  }
}

}  // namespace

extern "C" int cpu_rowsweep(int mode, const char* A0, const char* B0, size_t m, size_t n, size_t p, double g,
                            double h, int match, int mismatch, size_t rows, double* score, double* seconds) {
  if (!A0 || !B0 || m == 0 || n == 0 || p == 0 || rows > m) return -1;
  if (rows == 0) rows = m;
  const auto t0 = std::chrono::steady_clock::now();
  if (mode == 0) {
    const double NI = -std::numeric_limits<double>::infinity();
    std::vector<double> P1(n + 1, NI), P2(n + 1), P3(n + 1, NI), C1(n + 1), C2(n + 1), C3(n + 1);
    std::vector<double> omega(n + 1), part(n + 1);
    // row 0, start type -1 (:212-227, :259-280)
    P1[0] = 0;
    P2[0] = NI;
    for (size_t j = 1; j <= n; ++j) P2[j] = -h - g * (double)j;
    for (size_t i = 1; i <= rows; ++i) {
      C1[0] = NI;
      C2[0] = NI;
      C3[0] = -h - g * (double)i;
      map_blocks(n, p, [&](size_t s, size_t e) {  // ComputeRowMapThread13
        for (size_t j = s; j < e; ++j) {
          const double f = (A0[i - 1] == B0[j - 1]) ? 1.0 : 0.0;
          C1[j] = f + std::max(std::max(P1[j - 1], P2[j - 1]), P3[j - 1]);
          C3[j] = std::max(std::max(P1[j] - g - h, P2[j] - g - h), P3[j] - g);
        }
      });
      omega[0] = C2[0];
      map_blocks(n, p, [&](size_t s, size_t e) {  // ComputeOmegaMapThread
        for (size_t j = s; j < e; ++j) omega[j] = (double)j * g + std::max(C1[j - 1] - g - h, C3[j - 1] - g - h);
      });
      prefix_max(p, omega, part);
      map_blocks(n, p, [&](size_t s, size_t e) {  // ComputeRowMapThread2
        for (size_t j = s; j < e; ++j) C2[j] = part[j] - (double)j * g;
      });
      P1.swap(C1);
      P2.swap(C2);
      P3.swap(C3);
    }
    if (score) *score = std::max(std::max(P1[n], P2[n]), P3[n]);
  } else {
    const int32_t G = (int32_t)g;
    std::vector<int32_t> Hp(n + 1, 0), Hc(n + 1, 0), omega(n + 1), part(n + 1);
    int32_t best = 0;
    for (size_t i = 1; i <= rows; ++i) {
      map_blocks(n, p, [&](size_t s, size_t e) {  // phase 1: cells that depend on row i-1
        for (size_t j = s; j < e; ++j) {
          const int32_t sc = (A0[i - 1] == B0[j - 1]) ? match : mismatch;
          Hc[j] = std::max(0, std::max(Hp[j - 1] + sc, Hp[j] - G));
        }
      });
      omega[0] = 0;
      map_blocks(n, p, [&](size_t s, size_t e) {  // phase 2: omega
        for (size_t j = s; j < e; ++j) omega[j] = Hc[j] + (int32_t)j * G;
      });
      prefix_max(p, omega, part);
      map_blocks(n, p, [&](size_t s, size_t e) {  // phase 4: H
        for (size_t j = s; j < e; ++j) Hc[j] = part[j] - (int32_t)j * G;
      });
      Hc[0] = 0;
      for (size_t j = 1; j <= n; ++j) best = std::max(best, Hc[j]);
      Hp.swap(Hc);
    }
    if (score) *score = (double)best;
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  return 0;
}
