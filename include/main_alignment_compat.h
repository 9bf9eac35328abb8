/* main_alignment_compat.h -- the reference's alignment_algorithm/main_alignment.h API,
 * source- and binary-compatible, backed by the GPU.
 *
 * Replaces alignment_algorithm/main_alignment.h:11-38 of
 * D-2n/CSE305_Parallel_Sequence_Alignment: the same declarations (same types, so the
 * same C++ manglings) and the same include guard, so a translation unit compiled
 * against either header links against libmsa_compat.so, which defines them all:
 *
 *   main_alignment_function   (:38, main_alignment.cpp:353-410)  the single subproblem
 *       [(0,0,-1),(m,n,1)]: GPU fill + device find_alignment walk (msa_main_alignment);
 *       stdout "bp1\nbp1.2\nbp2\nbp3\nbp4\n" + print_seq's two lines, written atomically
 *       per call so concurrent callers (testing.cpp:145-158) do not interleave; returns 0.
 *   optimal_alignment         (:36, main_alignment.cpp:202-351)  every subproblem between
 *       consecutive partition points the reference solves (its three-round selection),
 *       concurrently on the GPU (msa_optimal_alignment), the reference's stitch (the
 *       link into the last subproblem is never made, :344-348) and print_seq; one atomic
 *       stdout write.  As in the definition (not the header's parameter names), the 4th
 *       and 5th arguments are m and n.
 *   OptimalAlignmentMapThread (:17, main_alignment.cpp:11-22)  one Subproblem on the GPU
 *       (msa_subproblem); prints bp1, bp1.2, bp2, bp3, bp4; begin/end = the malloc'd
 *       alignment_begin / alignment_end list (nodes are never freed, as the reference's).
 *   print_align               (:19, :26-31)   "(%ld, %ld, %d)\n" per node.
 *   print_seq                 (main_alignment.cpp:32-55, not in the reference header)
 *   ParallelPrefix, PrefixInitMapThread, PrefixSumMapThread   (:22-27, :65-156)
 *   ComputeOmegaMapThread, compute_omega_parallel, assign_processors   (:29-34, :158-200)
 *       the reference's subproblem scheduler bookkeeping (O(subproblems) integer work on
 *       the host; no DP cell).  ParallelPrefix returns the inclusive prefix sum it is
 *       written to compute; the reference's pointer-jumping threads race on the block
 *       sums (not idempotent for sums), so for more than one block its
 *       output can differ run to run -- this one is the race-free value.
 *       ComputeOmegaMapThread follows the header's signature (offset `long int`, m/n by
 *       position as the definition uses them).
 *
 * Unlike the reference, a failure (no gfx950 GPU, an empty or backward subproblem)
 * fails loudly: main_alignment_function prints the msa status to stderr and returns it;
 * the void functions throw std::runtime_error / std::invalid_argument.  Non-integral g/h
 * run the GPU double row sweep.  p only sizes the reference's thread counts. */
#pragma once
#ifndef main_alignment_H
#define main_alignment_H

#include <math.h>
#include <stdio.h>

#include <deque>
#include <thread>
#include <vector>

#include "subproblem_alignment_compat.h"

typedef struct parallel_prefix_queue_element {
  long int value;
  size_t begin_id;
  size_t end_id;
  struct parallel_prefix_queue_element* next;
} queue_indices;

void OptimalAlignmentMapThread(char* A, char* B, size_t m, size_t n, size_t ida, size_t idb, size_t p, int start_type,
                               int end_type, double g, double h, align*& begin, align*& end);

void print_align(align* begin);

void print_seq(char* A, char* B, align* begin);

void PrefixSumMapThread(std::vector<long int>& sums, long int value, queue_indices* curr);

void PrefixInitMapThread(std::vector<long int>& values, std::vector<long int>& sums, queue_indices& q);

void ParallelPrefix(size_t p, std::vector<long int>& values, std::vector<long int>& partial_sums);

void ComputeOmegaMapThread(std::vector<align>::iterator begin, std::vector<align>::iterator end, size_t n, size_t m,
                           size_t p, std::vector<long int>& omega, long int offset);

void compute_omega_parallel(std::vector<align>& partial_bp, size_t n, size_t m, size_t p, size_t len,
                            std::vector<long int>& omega);

size_t assign_processors(long int sum_prev, long int curr_subproblem);

void optimal_alignment(char* A, char* B, std::vector<align> partial_bp, size_t n, size_t m, size_t p, double g,
                       double h);

int main_alignment_function(char* A, char* B, size_t m, size_t n, size_t p, double g, double h);

#endif
