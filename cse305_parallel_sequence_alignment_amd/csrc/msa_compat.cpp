// msa_compat.cpp -- int main_alignment_function(...) with the reference's C++
// signature (alignment_algorithm/main_alignment.h:38), over the C-ABI.
// See include/main_alignment_compat.h for the contract.
#include <cstdio>
#include <mutex>
#include <vector>

#include "main_alignment_compat.h"
#include "msa.h"

namespace {
std::mutex g_stdout_mu;  // one call's lines stay together on stdout
}

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
  std::lock_guard<std::mutex> lk(g_stdout_mu);
  std::fwrite(text.data(), 1, len, stdout);
  std::fflush(stdout);
  return 0;
}
