// msa_types.h -- structs shared by the HIP kernels and the host side of the
// C-ABI (plain C layout, no torch types).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Algorithms the stripe kernel implements.
enum msa_alg {
  MSA_ALG_SWL = 0,   // Smith-Waterman, linear gap        (config C2, C4)
  MSA_ALG_SWA = 1,   // Smith-Waterman, affine gap        (config C5)
  MSA_ALG_NWA = 2,   // reference Gotoh, start type -1, h>=0, values only (banded, C3)
  MSA_ALG_REF = 3,   // reference Gotoh T1/T2/T3, any start type, exact -inf
  MSA_ALG_PART = 4,  // partial.cpp Gotoh with int32 wrap semantics
  MSA_ALG_SWL0 = 5,  // Smith-Waterman, linear gap, every substitution score >= 0 (plan's
                     // choice for MSA_SW_LINEAR when match, mismatch >= 0: no zero floor)
  MSA_ALG_REF1 = 6,  // reference Gotoh, start type -1 (main_alignment_function's subproblem),
                     // direction bytes: the tagged-max form of MSA_ALG_REF (msa_kernels.hip)
  MSA_ALG_SWLP = 7,  // MSA_ALG_SWL0 for TWO pairs per lane as packed int16 (batch, score only:
                     // pairs 2c and 2c+1 share rows/columns counts and the column sequence)
};

// Per-cell outputs.
enum msa_out {
  MSA_OUT_NONE = 0,  // scores only
  MSA_OUT_H = 1,     // int32 H per cell (skewed stripe layout)
  MSA_OUT_DIR = 2,   // uint8 traceback bits per cell (skewed stripe layout)
  MSA_OUT_TAB = 3,   // three int32 planes T1,T2,T3 per cell (skewed stripe layout)
};

// One pair of sequences inside a launch.  Codes are uint8 in [0,8).
typedef struct msa_pair_desc {
  int64_t a_off;       // offset of row codes (A[0] = row 1) in the A code array
  int64_t b_off;       // offset of column codes (B[0] = column 1) in the B code array
  int32_t m, n;        // rows, columns
  int32_t stripe0;     // first global stripe index of this pair (result / meta arrays)
  int32_t pmax;        // phases reserved per stripe in the output layout
  int64_t out_off;     // element offset of this pair's output block
  int64_t cod_off;     // byte offset of this pair's padded column-code segment in each code copy
} msa_pair_desc;

// Per-stripe metadata written by the kernel (host uses it to de-skew).
typedef struct msa_stripe_meta {
  int32_t cs;          // column processed by lane 0 at step 0 (lane r: cs + t - r)
  int32_t phases;      // phases the stripe ran
  int32_t best;        // SW: best H in the stripe (INT32_MIN if none)
  int32_t best_i;      // SW: row of the best (first max, row-major)
  int32_t best_j;      // SW: column of the best
  int32_t fin[3];      // global: state at (m, n) if this stripe holds row m
  int32_t has_fin;
  int32_t pad[3];
} msa_stripe_meta;

// Launch-wide scoring / geometry.
typedef struct msa_kparams {
  int32_t alg, out;
  int32_t match, mismatch;  // substitution (SW); REF: 1/0; PART: 0/1
  int32_t gap_open;         // SW: open cost (first gap char); REF/NWA/PART: g+h
  int32_t gap_ext;          // SW: extend cost;                REF/NWA/PART: g
  int32_t h;                // REF/NWA: h (border offsets)
  int32_t start_type;       // REF/PART start type
  int32_t band;             // -1: none, else |i-j| <= band
  int32_t single;           // 1: one pair split in groups of WAVES stripes over workgroups;
                            // 2: one banded pair in chunks of chunk_c stripes, one workgroup
                            //    per chunk, each started chunk_warm stripes early from a guess
                            //    (rank convergence, msa_kernels.hip)
  int32_t n_pairs;
  int32_t n_items;          // tickets
  uint32_t epoch;           // tag for cross-workgroup granules (nonzero, new per launch)
  int32_t sched_cap;        // stripes per item the LDS schedule can hold
  int32_t lds_code_bytes;   // per copy
  int32_t lds_row_words;    // wrap row buffer entries per carried value (batch mode)
  int32_t chunk_c;          // single == 2: stripes each chunk outputs
  int32_t chunk_warm;       // single == 2: warm-up stripes computed before a chunk's first one
  int32_t groups;           // single == 3 (a batch too small to fill the chip): items per pair (or
                            //   per packed couple), each W consecutive stripes, chained through
                            //   granules like single mode; every pair has the same m
  int32_t code_whole;       // flow kernels: 1 = every LDS code copy holds the whole row (no ring)
} msa_kparams;

#ifdef __cplusplus
}
#endif
