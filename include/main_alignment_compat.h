/* main_alignment_compat.h -- the reference's C++ entry point, re-exported.
 *
 * libmsa_compat.so defines, with C++ linkage (mangled
 * _Z23main_alignment_functionPcS_mmmdd), exactly the function the reference's
 * harness links:
 *
 *   int main_alignment_function(char* A, char* B, size_t m, size_t n, size_t p, double g, double h);
 *
 * declared at alignment_algorithm/main_alignment.h:38 and defined at
 * alignment_algorithm/main_alignment.cpp:353-410.  Same contract: A and B are
 * 1-based caller buffers (A[1..m], B[1..n]; element 0 is never read), nothing
 * is freed, stdout receives "bp1\nbp1.2\nbp2\nbp3\nbp4\n" and the two gapped
 * alignment lines (print_seq, main_alignment.cpp:32-55), written atomically
 * per call so concurrent callers (testing.cpp:145-158) do not interleave.
 * Returns 0 like the reference.  Unlike the reference it fails loudly instead
 * of computing on the CPU: on a machine without a gfx950 GPU, or for
 * parameters the GPU path does not take (non-integral g/h, m or n == 0), it
 * prints the msa status to stderr and returns that nonzero status.
 *
 * All DP cells are computed by the HIP stripe kernels in libmsa.so through
 * msa_main_alignment (include/msa.h). */
#ifndef MAIN_ALIGNMENT_COMPAT_H
#define MAIN_ALIGNMENT_COMPAT_H
#include <stddef.h>

int main_alignment_function(char* A, char* B, size_t m, size_t n, size_t p, double g, double h);

#endif
