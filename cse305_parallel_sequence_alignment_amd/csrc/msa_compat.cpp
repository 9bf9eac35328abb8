// msa_compat.cpp -- the reference's alignment_algorithm/main_alignment.h API with its C++
// signatures (include/main_alignment_compat.h), over the C-ABI of libmsa.so.  Every DP cell
// is computed by the HIP kernels (msa_main_alignment, msa_optimal_alignment, msa_subproblem);
// this file converts between the reference's types (char* 1-based buffers, std::vector<align>,
// malloc'd align lists, stdout) and the C-ABI, and restates the scheduler's bookkeeping
// helpers (omega, prefix sums, processor shares: main_alignment.cpp:65-200).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "main_alignment_compat.h"
#include "msa.h"

namespace {

std::mutex g_stdout_mu;  // one call's lines stay together on stdout

void emit(const char* text, size_t len) {
  std::lock_guard<std::mutex> lk(g_stdout_mu);
  std::fwrite(text, 1, len, stdout);
  std::fflush(stdout);
}

[[noreturn]] void fail(const char* fn, int rc) {
  const std::string msg = std::string(fn) + ": " + msa_status_string(rc) + " (status " + std::to_string(rc) + ")";
  if (rc == MSA_ERR_ARG) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

align* node(const msa_node& x, align* next) {
  align* a = (align*)std::malloc(sizeof(align));
  if (!a) throw std::bad_alloc();
  a->i = x.i;
  a->j = x.j;
  a->t = x.t;
  a->next = next;
  return a;
}

const char kProgress[] = "bp1\nbp1.2\nbp2\nbp3\nbp4\n";  // OptimalAlignmentMapThread's prints (:12-21)

}  // namespace

int main_alignment_function(char* A, char* B, size_t m, size_t n, size_t p, double g, double h) {
  // five progress lines + two alignment lines of at most m+n characters
  std::vector<char> text(64 + 2 * (m + n + 2));
  size_t len = 0;
  double score = 0.0;
  const int rc = msa_main_alignment(A, B, m, n, p, g, h, text.data(), text.size(), &len, &score);
  if (rc != MSA_OK) {
    std::fprintf(stderr, "main_alignment_function: %s (status %d)\n", msa_status_string(rc), rc);
    return rc;
  }
  emit(text.data(), len);
  return 0;
}

// main_alignment.cpp:11-22: Subproblem(A, B, m, n, ida, idb, p, start, end, g, h), compute_tables(),
// find_alignment(); begin / end = alignment_begin / alignment_end
void OptimalAlignmentMapThread(char* A, char* B, size_t m, size_t n, size_t ida, size_t idb, size_t p, int start_type,
                               int end_type, double g, double h, align*& begin, align*& end) {
  (void)p;
  std::vector<msa_node> nodes(m + n + 2);
  size_t cnt = 0;
  msa_node endn{};
  int inv = 0;
  const int rc = msa_subproblem(A, B, m, n, ida, idb, start_type, end_type, g, h, nullptr, nullptr, nullptr,
                                nodes.data(), nodes.size(), &cnt, &endn, &inv);
  if (rc != MSA_OK) fail("OptimalAlignmentMapThread", rc);
  if (cnt == 0) {  // find_alignment's loop never ran: alignment_begin = NULL (subproblem_alignment.cpp:170)
    begin = NULL;
    end = node(endn, NULL);
  } else {  // nodes[0 .. cnt) = alignment_begin .. alignment_end
    end = node(nodes[cnt - 1], NULL);
    align* cur = end;
    for (size_t k = cnt - 1; k-- > 0;) cur = node(nodes[k], cur);
    begin = cur;
  }
  emit(kProgress, sizeof(kProgress) - 1);
}

// main_alignment.cpp:26-31
void print_align(align* begin) {
  for (; begin != NULL; begin = begin->next) printf("(%ld, %ld, %d)\n", (long)begin->i, (long)begin->j, begin->t);
}

// main_alignment.cpp:32-55: A's characters where the node consumes A (t 1 or 3), B's where it
// consumes B (t 1 or 2), '-' elsewhere
void print_seq(char* A, char* B, align* begin) {
  std::string a, b;
  for (align* x = begin; x != NULL; x = x->next) {
    a += (x->t == 1 || x->t == 3) ? A[x->i] : '-';
    b += (x->t == 1 || x->t == 2) ? B[x->j] : '-';
  }
  a += '\n';
  a += b;
  a += '\n';
  emit(a.data(), a.size());
}

// main_alignment.cpp:65-71: add `value` to curr's block
void PrefixSumMapThread(std::vector<long int>& sums, long int value, queue_indices* curr) {
  if (curr == NULL) return;
  for (size_t i = curr->begin_id; i < curr->end_id; i++) sums[i] += value;
}

// main_alignment.cpp:73-79: the block's local inclusive prefix; q.value = its total
void PrefixInitMapThread(std::vector<long int>& values, std::vector<long int>& sums, queue_indices& q) {
  sums[q.begin_id] = values[q.begin_id];
  for (size_t i = q.begin_id + 1; i < q.end_id; i++) sums[i] = sums[i - 1] + values[i];
  q.value = sums[q.end_id - 1];
}

// main_alignment.cpp:81-156: partial_sums[i] = values[0] + ... + values[i] (the race-free value of
// the reference's block scan + pointer jumping; see the header)
void ParallelPrefix(size_t p, std::vector<long int>& values, std::vector<long int>& partial_sums) {
  if (p == 0) throw std::invalid_argument("ParallelPrefix: p = 0 (the reference divides by it)");
  const size_t n = values.size();
  if (partial_sums.size() < n) partial_sums.resize(n);
  long int run = 0;
  for (size_t i = 0; i < n; ++i) partial_sums[i] = run += values[i];
}

// main_alignment.cpp:158-167 (m, n by position as the definition uses them): omega of each
// subproblem [begin, begin+1) = max(ceil(di / (m/p)), ceil(dj / (n/p))) with the reference's size_t
// differences and double arithmetic
void ComputeOmegaMapThread(std::vector<align>::iterator begin, std::vector<align>::iterator end, size_t m, size_t n,
                           size_t p, std::vector<long int>& omega, long int offset) {
  size_t i = 0;
  for (; begin + 1 != end; ++begin, ++i) {
    const long int a = (long int)std::ceil(1.0 * ((begin + 1)->i - begin->i) / ((1.0 * m) / p));
    const long int b = (long int)std::ceil(1.0 * ((begin + 1)->j - begin->j) / ((1.0 * n) / p));
    omega[i + offset] = std::max(a, b);
  }
}

// main_alignment.cpp:169-190: the reference's thread blocks, run one after the other (their writes
// are disjoint, so the values are those of the threaded run)
void compute_omega_parallel(std::vector<align>& partial_bp, size_t m, size_t n, size_t p, size_t len,
                            std::vector<long int>& omega) {
  if (p == 0) throw std::invalid_argument("compute_omega_parallel: p = 0 (the reference divides by it)");
  size_t block = len / p, threads = p;
  if (p > len) {
    block = 1;
    threads = len;
  }
  if (threads == 0) throw std::length_error("compute_omega_parallel: no subproblems (the reference sizes workers(-1))");
  if (partial_bp.size() < (threads - 1) * block + 1)
    throw std::invalid_argument("compute_omega_parallel: len exceeds the partition");
  if (omega.size() < partial_bp.size() - 1) omega.resize(partial_bp.size() - 1);
  auto start = partial_bp.begin();
  for (size_t t = 0; t + 1 < threads; ++t, start += block)
    ComputeOmegaMapThread(start, start + block + 1, m, n, p, omega, (long int)(t * block));
  ComputeOmegaMapThread(start, partial_bp.end(), m, n, p, omega, (long int)((threads - 1) * block));
}

// main_alignment.cpp:192-200
size_t assign_processors(long int sum_prev, long int curr_subproblem) {
  if (sum_prev % 3 == 0) return (curr_subproblem + 2) / 3;
  if (sum_prev % 3 == 1) return 1 + curr_subproblem / 3;
  return 1 + (curr_subproblem + 1) / 3;
}

// main_alignment.cpp:202-351 (4th / 5th arguments = m, n as the definition uses them)
void optimal_alignment(char* A, char* B, std::vector<align> partial_bp, size_t m, size_t n, size_t p, double g,
                       double h) {
  std::vector<msa_node> bp(partial_bp.size());
  size_t span = 0;
  for (size_t k = 0; k < bp.size(); ++k) {
    bp[k] = msa_node{partial_bp[k].i, partial_bp[k].j, partial_bp[k].t, 0};
    if (k) span += (partial_bp[k].i - partial_bp[k - 1].i) + (partial_bp[k].j - partial_bp[k - 1].j) + 2;
  }
  // every solved subproblem's five progress lines + two alignment lines of at most the stitched path
  std::vector<char> text((sizeof(kProgress) - 1) * bp.size() + 2 * (span + 2) + 64);
  size_t len = 0;
  const int rc = msa_optimal_alignment(A, B, m, n, p, g, h, bp.data(), bp.size(), 0, text.data(), text.size(), &len,
                                       nullptr, 0, nullptr);
  if (rc != MSA_OK) fail("optimal_alignment", rc);
  emit(text.data(), len);
}
