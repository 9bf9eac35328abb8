/*
 * msa.h -- C-ABI of the MI355X-native pairwise-alignment library (libmsa.so).
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures; a
 * stream is passed as `void*` holding a hipStream_t, NULL = default stream).
 * Every function returns an msa_status (0 = OK, < 0 = error); nothing throws
 * across this boundary.  All compute runs in hand-written HIP kernels for
 * gfx950; there is no CPU fallback: without a usable GPU the calls return
 * MSA_ERR_NODEV.
 *
 * Reference interfaces each entry point replaces (D-2n/CSE305_Parallel_Sequence_Alignment):
 *   msa_main_alignment   int main_alignment_function(char*,char*,size_t,size_t,size_t,double,double)
 *                        alignment_algorithm/main_alignment.h:38, .cpp:353-410
 *                        (with OptimalAlignmentMapThread :11-22 and print_seq :32-55)
 *   msa_subproblem       class Subproblem ctor + compute_tables() + find_alignment()
 *                        alignment_algorithm/subproblem_alignment.h:36-74,
 *                        subproblem_alignment.cpp:329-355 (fill), :105-172 (traceback)
 *   msa_partial_partition findPartialBalancedPartitionParallel(...)
 *                        sequence_alignment/partial.h:41, partial.cpp:149-163
 *   msa_non_parallel_tables  Subproblem::non_parallel_tables(), subproblem_alignment.cpp:357-422
 *   msa_subproblem_f64   Subproblem ctor + compute_tables() in double for any g, h (:251-355)
 *   msa_subproblem_row   Subproblem::compute_row / *MapThread bodies (:212-327)
 *   msa_optimal_alignment optimal_alignment(...), main_alignment.h:34, main_alignment.cpp:158-351
 *   msa_main_alignment_partitioned  main_alignment_function with its commented-out
 *                        partition step (main_alignment.cpp:365,372) enabled
 *   msa_partial_tables   initializeTables/initializeReverseTables/fillTablesParallel/
 *                        fillReverseTablesParallel, partial.h:25-35, partial.cpp:13-79
 *   msa_partition_tables findPartitionParallel over caller tables, partial.h:37-39, partial.cpp:81-146
 *   msa_plan_*           device-resident batch / single-pair fills (build extension:
 *                        configs C2-C5 of BASELINE.json; no reference counterpart,
 *                        same cell recurrence family as subproblem_alignment.cpp:396-398)
 */
#ifndef MSA_H
#define MSA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------ */
typedef enum msa_status {
  MSA_OK = 0,
  MSA_ERR_ARG = -1,          /* bad argument (size 0 where the path needs >0, NULL, ...) */
  MSA_ERR_ALPHABET = -2,     /* more than 8 distinct symbols in a pair */
  MSA_ERR_HIP = -3,          /* a HIP runtime call failed */
  MSA_ERR_NODEV = -4,        /* no gfx950 device visible */
  MSA_ERR_UNSUPPORTED = -5,  /* e.g. non-integral g/h (the GPU path is exact int32) */
  MSA_ERR_TIMEOUT = -6,      /* a cross-workgroup wait exceeded its bound */
  MSA_ERR_NOMEM = -7,
  MSA_ERR_CAPACITY = -8,     /* caller buffer too small */
  MSA_ERR_NOMATCH = -9       /* traceback found no predecessor (cannot happen for integral g,h) */
} msa_status;

const char* msa_status_string(int status);
int msa_version(void);
/* number of usable gfx950 devices */
int msa_device_count(int* count);

/* Admission control of the host-pointer entry points (msa_main_alignment, msa_subproblem,
 * msa_partial_*, msa_sw_align, msa_optimal_alignment's subproblems).  The reference's callers
 * run main_alignment_function from hardware_concurrency threads at once on whole sequences
 * (test_functions/testing.cpp:269-280 and :352-358, calls at :261 and :345); every call here
 * reserves its estimated device footprint against a per-device budget before allocating and
 * waits (FIFO) until it fits, instead of failing with MSA_ERR_NOMEM.  A call larger than the
 * budget runs alone.  Budget: env MSA_DEVICE_BUDGET_MB, else 90% of device memory;
 * msa_set_device_budget(bytes) sets it for the current device (0 = back to the default).
 * msa_device_budget_info: out5 = {budget, bytes admitted now, peak admitted bytes since the
 * last set, calls that had to wait, calls admitted}. */
int msa_set_device_budget(int64_t bytes);
int msa_device_budget_info(int64_t* out5);
/* Memory held on the current device: out4 = {bytes admitted now, idle cached plans of the
 * reference walk (footprint estimate), free blocks of the device pool, admissions that released
 * the idle ones first}.  An admission that would put admitted + idle bytes over the budget first
 * destroys the idle cached plans and frees the pool's blocks.  Plans created directly through
 * msa_plan_create (the device-resident API below) are the caller's and are not admitted. */
int msa_device_memory_info(int64_t* out4);

/* Node of an alignment path: the reference's `align` struct
 * (subproblem_alignment.h:8-13) without the `next` pointer. */
typedef struct msa_node {
  uint64_t i;
  uint64_t j;
  int32_t t;
  int32_t pad;
} msa_node;

/* ---- reference-compatible host-pointer entry points ---------------------
 * Character arrays follow the reference's conventions: A1/B1 are 1-based
 * (A1[0] never read), compared for equality only. */

/* main_alignment_function: writes the exact stdout text the reference prints
 * ("bp1".."bp4" then print_seq's two lines) into `text` (NUL-terminated),
 * *text_len = its length.  *score = max(T1,T2,T3)[m][n] (not exposed by the
 * reference; returned for convenience).  p only sets the reference's thread
 * count and is accepted for signature parity. */
int msa_main_alignment(const char* A1, const char* B1, size_t m, size_t n, size_t p, double g, double h,
                       char* text, size_t text_cap, size_t* text_len, double* score);

/* Subproblem(A1,B1,m,n,idA,idB,p,start,end,g,h) -> compute_tables(), and when
 * nodes != NULL, find_alignment().  After the constructor's swap (m > n) the
 * tables are (m'+1) x (n'+1), m' = min(m,n); T1/T2/T3 (each NULL or
 * (m'+1)*(n'+1) int32, row-major) receive the tables with INT32_MIN standing
 * for -infinity.  nodes[0..*n_nodes) = alignment_begin .. alignment_end;
 * *end_node = alignment_end; *invert = the constructor's swap flag. */
int msa_subproblem(const char* A1, const char* B1, size_t m, size_t n, size_t idA, size_t idB, int start_type,
                   int end_type, double g, double h, int32_t* T1, int32_t* T2, int32_t* T3, msa_node* nodes,
                   size_t nodes_cap, size_t* n_nodes, msa_node* end_node, int* invert);

/* Subproblem::non_parallel_tables (subproblem_alignment.cpp:357-422): the
 * tables of msa_subproblem printed as the reference prints them ("T1:" then
 * one line per row of "%lf " cells, -inf as "-inf"; then T2, T3) into `text`
 * (NUL-terminated; *text_len = its length; text may be NULL to size it). */
int msa_non_parallel_tables(const char* A1, const char* B1, size_t m, size_t n, size_t idA, size_t idB,
                            int start_type, int end_type, double g, double h, char* text, size_t text_cap,
                            size_t* text_len);

/* The reference's tables in IEEE double for ANY g, h (the int32 entry points
 * need integral g, h): Subproblem ctor + compute_tables
 * (subproblem_alignment.h:36-74, .cpp:329-355) as its row sweep -- T1/T3
 * elementwise, T2 by omega + inclusive prefix max (:229-326) -- on the GPU,
 * with the same double operations in the same order (bit-identical cells).
 * T1/T2/T3: (m'+1) x (n'+1) row-major doubles (-inf as -infinity), m' =
 * min(m,n) after the constructor's swap (*invert).  m = n = 0 is MSA_ERR_ARG.
 * mode MSA_F64_NON_PARALLEL computes T2 by non_parallel_tables' direct
 * recurrence (:398) instead -- the same values for integral g, h; for others
 * the two forms round differently, and each mode matches its reference twin. */
enum { MSA_F64_COMPUTE_TABLES = 0, MSA_F64_NON_PARALLEL = 1 };
int msa_subproblem_f64(const char* A1, const char* B1, size_t m, size_t n, size_t idA, size_t idB, int start_type,
                       double g, double h, int mode, double* T1, double* T2, double* T3, int* invert);

/* One step of the reference's row sweep on the GPU (double, bit-identical),
 * for the source-compatible Subproblem's compute_row and MapThread bodies:
 *   MSA_ROW_ZERO  compute_row(0)                  subproblem_alignment.cpp:259-280 (cur = row 0)
 *   MSA_ROW_FULL  compute_row(i > 0)              :282-326 (up = row i-1, cur = row i; vec optional)
 *   MSA_ROW_FIRST ComputeFirstRowMapThread         :212-227 on cur, columns [start, end)
 *   MSA_ROW_13    ComputeRowMapThread13            :229-235 up -> cur T1/T3, columns [start, end)
 *   MSA_ROW_OMEGA ComputeOmegaMapThread            :237-242 cur T1/T3 -> vec[start, end)
 *   MSA_ROW_T2    ComputeRowMapThread2             :244-249 vec -> cur T2, columns [start, end)
 * A1/B1 with idA/idB as the Subproblem holds them (after its swap); rows are
 * n+1 doubles; column ranges need 1 <= start <= end <= n+1. */
enum { MSA_ROW_FIRST = 1, MSA_ROW_13 = 2, MSA_ROW_OMEGA = 4, MSA_ROW_T2 = 8, MSA_ROW_ZERO = 16, MSA_ROW_FULL = 32 };
int msa_subproblem_row(int part, const char* A1, const char* B1, size_t idA, size_t idB, size_t n, size_t i,
                       int start_type, double g, double h, size_t start, size_t end, const double* up1,
                       const double* up2, const double* up3, double* cur1, double* cur2, double* cur3, double* vec);

/* optimal_alignment(A, B, partial_bp, m, n, p, g, h) (main_alignment.h:34,
 * main_alignment.cpp:202-351): solves the subproblems between consecutive
 * partition points bp[k] -> bp[k+1] (start type bp[k].t, end type -bp[k+1].t)
 * on the GPU, concurrently, in the reference's selection (with 2 or 3
 * subproblems only subproblem 0 is solved, :237-279), stitches their node
 * lists as :344-348 does (the link into the last subproblem is never made) and
 * writes the stdout text: "bp1".."bp4" per solved subproblem, then print_seq's
 * two lines.  flags = MSA_OPT_FIX_ALL solves and links every subproblem.
 * path (may be NULL) receives the stitched node list.  p only sizes the
 * reference's thread counts (omega / ParallelPrefix / assign_processors,
 * :158-200) and is accepted for signature parity.  Partition points must be
 * non-decreasing in i and j and inside [0,m] x [0,n]; a 0 x 0 subproblem is
 * MSA_ERR_ARG (the reference crashes on both). */
enum { MSA_OPT_FIX_ALL = 1 };
int msa_optimal_alignment(const char* A1, const char* B1, size_t m, size_t n, size_t p, double g, double h,
                          const msa_node* bp, size_t n_bp, int flags, char* text, size_t text_cap, size_t* text_len,
                          msa_node* path, size_t path_cap, size_t* n_path);

/* main_alignment_function with the partition step the reference leaves
 * commented out (main_alignment.cpp:365,372): the GPU partition
 * findPartialBalancedPartitionParallel(A1+1, B1+1, m, n, p, g, h, -1, -1)
 * (partial.cpp reads A[i-1], so it gets the 0-based view) feeding
 * msa_optimal_alignment.  Same text contract as msa_main_alignment. */
int msa_main_alignment_partitioned(const char* A1, const char* B1, size_t m, size_t n, size_t p, double g,
                                   double h, int flags, char* text, size_t text_cap, size_t* text_len);

/* findPartialBalancedPartitionParallel (partial.cpp:149-163), int32 wrap
 * semantics; A0/B0 are 0-based (partial.cpp reads A[i-1]).  out receives the
 * p+1 sorted partition points. */
int msa_partial_partition(const char* A0, const char* B0, size_t m, size_t n, size_t p, double g, double h,
                          int start_type, int end_type, msa_node* out, size_t cap, size_t* n_out);

/* The six int32 tables partial.cpp builds: T* (m+1)x(n+1), R* (m+2)x(n+2),
 * row-major; any pointer may be NULL. */
int msa_partial_tables(const char* A0, const char* B0, size_t m, size_t n, double g, double h, int start_type,
                       int end_type, int32_t* T1, int32_t* T2, int32_t* T3, int32_t* R1, int32_t* R2, int32_t* R3);

/* findPartitionParallel(T1, T2, T3, TR1, TR2, TR3, m, n, p, h) (partial.h:37-39,
 * partial.cpp:81-146) over tables the caller already holds: T* (m+1)x(n+1) and
 * TR* (m+2)x(n+2) int32, row-major, as partial.cpp's own fills leave them.  The
 * band maxima run on the GPU (int32 wrap, first maximum in the reference's scan
 * order); out receives the p+1 points sorted as partial.cpp:141-143. */
int msa_partition_tables(const int32_t* T1, const int32_t* T2, const int32_t* T3, const int32_t* R1,
                         const int32_t* R2, const int32_t* R3, size_t m, size_t n, size_t p, double h,
                         msa_node* out, size_t cap, size_t* n_out);

/* ---- device-resident plans (configs C2-C5) --------------------------------
 * A plan owns the device scratch for one shape of work; running it launches
 * the stripe kernel + a tiny per-pair reduction on `stream` (no allocation,
 * no host sync inside msa_plan_run).  Inputs are uint8 codes in [0,8) already
 * in device memory (see msa_encode_pair for the host-side code map); the
 * Smith-Waterman algorithms reserve code 7 (out-of-matrix sentinel), so their
 * inputs use codes 0..6. */
typedef enum msa_alg_e {
  MSA_SW_LINEAR = 0,  /* Smith-Waterman, linear gap (gap_open == gap_extend used) */
  MSA_SW_AFFINE = 1,  /* Smith-Waterman, affine gap */
  MSA_NW_BANDED = 2,  /* reference Gotoh (g=gap_extend, h=gap_open-gap_extend), start type -1, optional band */
  MSA_REF_GOTOH = 3,  /* reference Gotoh T1/T2/T3, any start type, exact -inf */
  MSA_PARTIAL = 4     /* partial.cpp forward Gotoh, int32 wrap */
} msa_alg_e;

typedef enum msa_out_e { MSA_CELLS_NONE = 0, MSA_CELLS_H = 1, MSA_CELLS_DIR = 2, MSA_CELLS_TAB = 3 } msa_out_e;

typedef struct msa_plan_desc {
  int32_t alg;         /* msa_alg_e */
  int32_t cells;       /* msa_out_e */
  int32_t match, mismatch;
  int32_t gap_open;    /* SW: cost of the first gap char; Gotoh: g + h */
  int32_t gap_extend;  /* SW: each further gap char; Gotoh: g */
  int32_t start_type;  /* MSA_REF_GOTOH / MSA_PARTIAL */
  int32_t band;        /* MSA_NW_BANDED: |i-j| <= band, -1 = none */
  int32_t track_end;   /* SW: also report the end cell (first max, row-major) */
  int32_t single;      /* 1: one pair spread over many workgroups; 0: one workgroup per pair */
  int64_t n_pairs;
  const int64_t* m;    /* host arrays, n_pairs each */
  const int64_t* n;
  const int64_t* a_off; /* offsets of each pair's row / column codes in the device arrays */
  const int64_t* b_off;
} msa_plan_desc;

typedef struct msa_pair_result {
  int32_t score;
  int32_t status;
  int64_t end_i, end_j;  /* SW: end cell; Gotoh: (m, n) */
  int32_t fin[3];        /* Gotoh: state at (m, n) (T1,T2,T3 / H,E,F) */
  int32_t pad;
} msa_pair_result;

typedef struct msa_plan msa_plan;

int msa_plan_create(const msa_plan_desc* desc, msa_plan** plan);
void msa_plan_destroy(msa_plan* plan);
/* Elements (int32 for H/TAB planes, bytes for DIR) the per-cell output needs. */
int msa_plan_cells_size(const msa_plan* plan, int64_t* elems);
/* Launch on `stream`.  dA/dB: device code arrays.  cells0..2: device output
 * (H: cells0; DIR: cells0 as uint8; TAB: three planes), may be NULL for NONE. */
int msa_plan_run(msa_plan* plan, const uint8_t* dA, const uint8_t* dB, void* cells0, void* cells1, void* cells2,
                 void* stream);
/* Copy per-pair results to the host (synchronizes `stream`).  Returns
 * MSA_ERR_TIMEOUT if any run since the plan was created (or since the last
 * msa_plan_clear_error) had a kernel wait hit its spin limit: the plan's error
 * word is sticky, so one check after many runs covers all of them. */
int msa_plan_results(msa_plan* plan, msa_pair_result* out, void* stream);
/* How the last run was computed: out4 = {launch mode (0 stripe kernel, 1 two-pass
 * flow kernel, 2 chunked banded), chunks, converged (chunked: 1 = every chunk
 * converged and the cells came from the chunk launch, 0 = the exact single-mode
 * launch recomputed them; -1 otherwise), warm-up stripes per chunk | 1 << 16 when
 * chunks >= 1 wrote int16 cells widened by the chunk constants' add}.
 * Synchronizes `stream` for mode 2. */
int msa_plan_run_info(msa_plan* plan, int32_t* out4, void* stream);
/* How the plan launches (for tests and tools): out8 = {mode: 0 stripe_kernel (batch), 1 flow_kernel
 * (single pair, two-pass), 2 chunked banded stripe_kernel, 3 split batch (every pair split into items
 * over several CUs), 4 band_kernel exact chain, 5 band_kernel chunked, 6 cflow_kernel (packed score-only
 * batch as flag-synchronised chains); workgroups of the main launch;
 * threads per workgroup; dynamic LDS bytes; flow pass-1 workgroups; workgroups of the separate pass-2
 * launch (flow_fill_kernel, long pairs; 0 = pass 2 runs inside the main launch); rows per lane;
 * items}. */
int msa_plan_launch_info(const msa_plan* plan, int32_t* out8);
/* The sticky error word (0 = no error; else the kernel site code), synchronizes. */
int msa_plan_error(msa_plan* plan, int* code, void* stream);
/* Reset the sticky error word (stream-ordered). */
int msa_plan_clear_error(msa_plan* plan, void* stream);
/* Per-pair scores of the last run into a device int32 array of n_pairs
 * (device-to-device copy on `stream`, no host sync): the input of a score
 * all-gather across ranks. */
int msa_plan_scores(msa_plan* plan, int32_t* d_scores, void* stream);
/* Per-stripe metadata (cs, phases ...) of the last run: 12 int32 per stripe. */
int msa_plan_stripe_meta(msa_plan* plan, int32_t* out, int64_t cap_stripes, void* stream);
int64_t msa_plan_stripes(const msa_plan* plan);
/* Layout of one pair's cells in the skewed output: out4 = {first stripe index
 * in the meta array, pmax (16-step blocks per stripe), element offset of the
 * pair's block, DP steps per kernel phase | R << 16}.  R = rows per lane
 * (0 means 1).  Cell (i, j) of stripe s = (i-1)/(64R), lane r = ((i-1)%(64R))/R,
 * row rho = (i-1)%R, step t = j - cs_s + r lives at element
 * out_off + ((s*pmax*4 + t/4)*R + rho)*256 + r*4 + t%4 (DIR bytes, R = 1:
 * (s*pmax + t/16)*1024 + r*16 + t%16), cs_s = meta[12*(stripe0+s)].  R = 2 only
 * for two-pass single-pair SW-linear H plans. */
int msa_plan_pair_layout(const msa_plan* plan, int64_t pair, int64_t* out4);
/* Smith-Waterman traceback ON THE DEVICE (msa_traceback.hip), for an
 * MSA_SW_AFFINE plan with MSA_CELLS_DIR after msa_plan_run on the same stream:
 * one workgroup (a walker wave, four stripe-group loader waves, an op decoder
 * wave) walks pair `pair`'s direction bytes dDir from the end cell the run
 * found (first maximum, row-major) and writes the ops end -> start into d_ops
 * ('M' diagonal, 'D' gap consuming B, 'I' gap consuming A; at most ops_cap,
 * m+n suffices) and d_info[8] = {n_ops, beg_i, beg_j, status, stripes
 * entered, groups staged on demand, s_memtime ticks of the walk, times the
 * walker waited for a loader} (beg = the first aligned cell, 1-based; status
 * 0, MSA_ERR_CAPACITY or MSA_ERR_TIMEOUT).  Asynchronous,
 * no host sync; tie order of the oracle's orc_sw. */
int msa_plan_traceback(msa_plan* plan, int64_t pair, const uint8_t* dDir, uint8_t* d_ops, int64_t ops_cap,
                       int64_t* d_info, void* stream);
/* Subproblem::find_alignment ON THE DEVICE (replaces the host walk over the
 * reference's T1/T2/T3 tables, subproblem_alignment.cpp:105-172) for an
 * MSA_REF_GOTOH plan with MSA_CELLS_DIR, after msa_plan_run on the same stream:
 * one wave starts at (m, n) in the table the reference's end rule picks for
 * end_type (:112-146, from the run's final state; end_type in {-3..-1, 1..3})
 * and walks the direction bytes until i == 0 or j == 0 (:147).  d_ops receives
 * one op per step, end -> start: the table the step leaves ('M' T1 / diagonal,
 * 'D' T2 / consumes B, 'I' T3 / consumes A; at most ops_cap, m+n suffices);
 * d_info[8] as msa_plan_traceback, with {n_ops, i+1, j+1, status} where (i, j)
 * is the border cell the walk stopped at and status 0, MSA_ERR_CAPACITY or
 * MSA_ERR_NOMATCH.  The reference's align nodes (coordinates, quirks Q1/Q2)
 * follow from the ops on the host in O(m+n) (msa_main_alignment does this). */
int msa_plan_traceback_gotoh(msa_plan* plan, int64_t pair, int end_type, const uint8_t* dDir, uint8_t* d_ops,
                             int64_t ops_cap, int64_t* d_info, void* stream);
/* Order-independent digest of pair `pair`'s H cells (oracle orc_checksum_h). */
int msa_plan_checksum(msa_plan* plan, const int32_t* dH, int64_t pair, uint64_t* digest, void* stream);
/* Device time (ms) of the last msa_plan_run's stripe kernel, from HIP events
 * recorded on the run's stream (synchronizes).  MSA_ERR_ARG if that run had
 * timing off. */
int msa_plan_last_kernel_ms(msa_plan* plan, float* ms);
/* Record the timing events in msa_plan_run (default on); off saves two stream
 * commands per run. */
int msa_plan_set_timing(msa_plan* plan, int on);

/* Map the symbols of a pair to codes 0..7 (equality preserved, first-seen
 * order).  Returns MSA_ERR_ALPHABET for more than 8 distinct symbols. */
int msa_encode_pair(const char* A0, size_t m, const char* B0, size_t n, uint8_t* codesA, uint8_t* codesB);

/* Host-pointer Smith-Waterman (build extension): score, end cell (first max
 * in row-major order) and, when cigar != NULL, the traceback as a run-length
 * M/I/D string (I consumes A, D consumes B) with its start cell.  At most 7
 * distinct symbols (MSA_ERR_ALPHABET otherwise). */
int msa_sw_align(const char* A0, size_t m, const char* B0, size_t n, int32_t match, int32_t mismatch,
                 int32_t gap_open, int32_t gap_extend, int32_t* score, int64_t* end_i, int64_t* end_j,
                 int64_t* beg_i, int64_t* beg_j, char* cigar, size_t cigar_cap);

#ifdef __cplusplus
}
#endif

#endif /* MSA_H */
