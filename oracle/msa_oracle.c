/*
 * msa_oracle.c -- CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library, the C++
 * drop-in layer, the Python package) links, loads or calls this file.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Parity pinning: every function below was checked against golden vectors
 * produced by the reference's own sources compiled unmodified from
 * /root/reference (oracle/Makefile -> oracle/_ref/libref.so, generator
 * tests/golden/make_golden.py).  See DESIGN.md "Oracle".
 *
 * Functions and the reference code each one restates:
 *   orc_subproblem_tables  subproblem_alignment.h:36-74 (ctor, A/B swap),
 *                          subproblem_alignment.cpp:357-399 (non_parallel_tables,
 *                          bit-identical to compute_tables :329-332, borders
 *                          :212-227, :259-292)
 *   orc_subproblem_traceback subproblem_alignment.cpp:105-172 (find_alignment,
 *                          tie order, quirks Q1 (:147,:170) and Q2 (:151))
 *   orc_print_seq          main_alignment.cpp:32-55
 *   orc_main_alignment     main_alignment.cpp:11-22 (OptimalAlignmentMapThread),
 *                          :202-351 (single-subproblem path), :353-410
 *   orc_main_alignment_dir the same path for integral g, h in 1 B/cell (direction
 *                          bytes + int64 rows) for the callers' whole-sequence sizes
 *                          (testing.cpp:261,345); equals orc_main_alignment
 *   orc_optimal_alignment  main_alignment.cpp:202-351 (subproblem selection of the
 *                          three rounds :232-341, stitch :344-348 incl. the
 *                          never-made link into the last subproblem), :32-55
 *   orc_partial_tables / orc_partial_partition
 *                          partial.cpp:9-163 with two's-complement wrap (the
 *                          reference's -O0 behaviour)
 *   orc_sw                 build extension (Smith-Waterman local, affine/linear),
 *                          "reference-anchored": same cell recurrence family
 *   orc_banded_ref         build extension: reference Gotoh (T1/T2/T3) restricted
 *                          to |i-j| <= w; equals orc_subproblem_tables when w >= max(m,n)
 *   orc_checksum_h         order-independent 64-bit digest of an int32 matrix
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR_ARG -1
#define ORC_ERR_CAP -2
#define ORC_ERR_NOMATCH -3 /* reference would read an uninitialised node (non-integral g/h) */
#define ORC_ERR_NOMEM -4

typedef struct {
  uint64_t i;
  uint64_t j;
  int32_t t;
  int32_t pad;
} orc_node;

static inline double dmax(double a, double b) { return a > b ? a : b; }
/* std::max(a,b) returns a when !(a < b): for the values here (no NaN) the
 * value is the same as dmax, which is all that matters. */

/* ---------------------------------------------------------------------------
 * Reference Subproblem: tables.
 *   A, B: the caller's 1-based arrays (A[0] never read).
 *   After the constructor's swap (m > n -> swap), tables are (m'+1) x (n'+1),
 *   row-major, row stride n'+1.  *invert reports whether the swap happened.
 * ------------------------------------------------------------------------- */
int orc_subproblem_tables(const char* A_in, const char* B_in, uint64_t m_in, uint64_t n_in,
                          uint64_t idA_in, uint64_t idB_in, int start_type, double g, double h,
                          double* T1, double* T2, double* T3, int* invert) {
  const char *A, *B;
  uint64_t m, n, idA, idB;
  if (m_in <= n_in) {
    A = A_in; B = B_in; m = m_in; n = n_in; idA = idA_in; idB = idB_in; *invert = 0;
  } else {
    A = B_in; B = A_in; m = n_in; n = m_in; idA = idB_in; idB = idA_in; *invert = 1;
  }
  const uint64_t W = n + 1;
  const double NI = -INFINITY;
#define T(tab, i, j) tab[(uint64_t)(i) * W + (j)]
  /* row 0: compute_row(0), subproblem_alignment.cpp:259-280 */
  T(T1, 0, 0) = NI; T(T2, 0, 0) = NI; T(T3, 0, 0) = NI;
  if (start_type == 1 || start_type == -1) T(T1, 0, 0) = 0;
  else if (start_type == -2) T(T2, 0, 0) = 0;
  else if (start_type == -3) T(T3, 0, 0) = 0;
  for (uint64_t j = 1; j <= n; j++) { /* ComputeFirstRowMapThread :212-227 */
    T(T1, 0, j) = NI;
    T(T3, 0, j) = NI;
    if (start_type == -2) T(T2, 0, j) = -g * (double)j;
    else if (start_type == 1 || start_type == 3) T(T2, 0, j) = NI;
    else T(T2, 0, j) = -h - g * (double)j;
  }
  for (uint64_t i = 1; i <= m; i++) {
    T(T1, i, 0) = NI; T(T2, i, 0) = NI; /* :282-292 */
    if (start_type == -3) T(T3, i, 0) = -g * (double)i;
    else if (start_type == 1 || start_type == 2) T(T3, i, 0) = NI;
    else T(T3, i, 0) = -h - g * (double)i;
    const char a = A[idA + i];
    for (uint64_t j = 1; j <= n; j++) { /* :396-398 */
      const double f = (a == B[idB + j]) ? 1.0 : 0.0;
      T(T1, i, j) = f + dmax(dmax(T(T1, i - 1, j - 1), T(T2, i - 1, j - 1)), T(T3, i - 1, j - 1));
      T(T3, i, j) = dmax(dmax(T(T1, i - 1, j) - g - h, T(T2, i - 1, j) - g - h), T(T3, i - 1, j) - g);
      T(T2, i, j) = dmax(dmax(T(T1, i, j - 1) - g - h, T(T2, i, j - 1) - g), T(T3, i, j - 1) - g - h);
    }
  }
  return ORC_OK;
}

/* ---------------------------------------------------------------------------
 * Reference Subproblem::find_alignment (subproblem_alignment.cpp:105-172).
 *   Works on the (already swapped) problem: A,B,m,n,idA,idB are the values the
 *   Subproblem object holds after its constructor.
 *   nodes[0..*n_nodes) = the list from alignment_begin to alignment_end.
 *   end_node receives alignment_end (always written).
 * ------------------------------------------------------------------------- */
int orc_subproblem_traceback(const char* A, const char* B, uint64_t m, uint64_t n, uint64_t idA,
                             uint64_t idB, int end_type, double g, double h, const double* T1,
                             const double* T2, const double* T3, orc_node* nodes, uint64_t cap,
                             uint64_t* n_nodes, orc_node* end_node) {
  const uint64_t W = n + 1;
  uint64_t i = m, j = n;
  orc_node cur;
  /* h_prime, subproblem_alignment.h:91-96 */
#define HPRIME(k) (((k) == end_type && end_type <= -2) ? h : 0.0)
  if (end_type > 0) {
    cur.t = end_type;
    if (end_type == 1) { cur.i = i + idA; cur.j = j + idB; }
    else if (end_type == 2) { cur.i = 0; cur.j = j + idB; }
    else { cur.i = i + idA; cur.j = 0; }
  } else {
    const double t1 = T(T1, m, n);
    const double t2 = T(T2, m, n) + HPRIME(-2);
    const double t3 = T(T3, m, n) + HPRIME(-3);
    if (t1 >= t2 && t1 >= t3) { cur.t = 1; cur.i = i + idA; cur.j = j + idB; }
    else if (t2 >= t1 && t2 >= t3) { cur.t = 2; cur.i = 0; cur.j = j + idB; }
    else { cur.t = 3; cur.i = i + idA; cur.j = 0; }
  }
  cur.pad = 0;
  *end_node = cur;
  /* The reference prepends nodes while walking back; we collect them in
   * reverse and flip at the end.  The final list skips the last-created node
   * (Q1: alignment_begin = curr_point->next). */
  uint64_t cnt = 0; /* number of created nodes, including the end node */
  /* worst case path length m+n+1 */
  orc_node* tmp = (orc_node*)malloc(sizeof(orc_node) * (m + n + 2));
  if (!tmp) return ORC_ERR_NOMEM;
  tmp[cnt++] = cur;
  int ct = cur.t;
  while (i > 0 && j > 0) {
    orc_node nw;
    nw.pad = 0;
    const char a = A[idA + i];
    const double f = (a == B[idB + j]) ? 1.0 : 0.0;
    if (ct == 1) {
      const double v = T(T1, i, j);
      if (v == f + T(T1, i - 1, j - 1)) { nw.t = 1; nw.i = i - 1 + idA; nw.j = j - 1 + idA; } /* Q2 */
      else if (v == f + T(T2, i - 1, j - 1)) { nw.t = 2; nw.i = 0; nw.j = j - 1 + idB; }
      else if (v == f + T(T3, i - 1, j - 1)) { nw.t = 3; nw.i = i - 1 + idA; nw.j = 0; }
      else { free(tmp); return ORC_ERR_NOMATCH; }
      i--; j--;
    } else if (ct == 2) {
      const double v = T(T2, i, j);
      if (v == -g - h + T(T1, i, j - 1)) { nw.t = 1; nw.i = i + idA; nw.j = j - 1 + idB; }
      else if (v == -g + T(T2, i, j - 1)) { nw.t = 2; nw.i = 0; nw.j = j - 1 + idB; }
      else if (v == -g - h + T(T3, i, j - 1)) { nw.t = 3; nw.i = i + idA; nw.j = 0; }
      else { free(tmp); return ORC_ERR_NOMATCH; }
      j--;
    } else {
      const double v = T(T3, i, j);
      if (v == -g - h + T(T1, i - 1, j)) { nw.t = 1; nw.i = i - 1 + idA; nw.j = j + idB; }
      else if (v == -g - h + T(T2, i - 1, j)) { nw.t = 2; nw.i = 0; nw.j = j + idB; }
      else if (v == -g + T(T3, i - 1, j)) { nw.t = 3; nw.i = i - 1 + idA; nw.j = 0; }
      else { free(tmp); return ORC_ERR_NOMATCH; }
      i--;
    }
    ct = nw.t;
    tmp[cnt++] = nw;
  }
#undef HPRIME
  /* list = tmp[cnt-2], tmp[cnt-3], ..., tmp[0]  (tmp[cnt-1] dropped) */
  const uint64_t len = cnt - 1;
  *n_nodes = len;
  if (len > cap) { free(tmp); return ORC_ERR_CAP; }
  for (uint64_t k = 0; k < len; k++) nodes[k] = tmp[cnt - 2 - k];
  free(tmp);
  return ORC_OK;
}
#undef T

/* main_alignment.cpp:32-55.  out1/out2 receive len chars + NUL.  Indices past
 * the caller's buffers (only possible in the reference's m>n quirk Q3) print '?'
 * here; the reference reads out of bounds there. */
void orc_print_seq(const char* A, const char* B, uint64_t lenA, uint64_t lenB, const orc_node* nodes,
                   uint64_t len, char* out1, char* out2) {
  for (uint64_t k = 0; k < len; k++) {
    const orc_node* p = &nodes[k];
    out1[k] = (p->t == 1 || p->t == 3) ? (p->i <= lenA ? A[p->i] : '?') : '-';
    out2[k] = (p->t == 1 || p->t == 2) ? (p->j <= lenB ? B[p->j] : '?') : '-';
  }
  out1[len] = 0;
  out2[len] = 0;
}

/* The observable output of main_alignment_function(A,B,m,n,p,g,h) for the live
 * single-subproblem partition [(0,0,-1),(m,n,1)]: "bp1".."bp4" from
 * OptimalAlignmentMapThread, then print_seq's two lines.  p only changes the
 * reference's thread count (bit-identical results), so it is not an input.
 * Writes the text (NUL-terminated) into out; returns bytes written or <0. */
int64_t orc_main_alignment(const char* A, const char* B, uint64_t m, uint64_t n, double g, double h,
                           char* out, uint64_t cap, double* score) {
  int inv;
  const uint64_t mm = m <= n ? m : n, nn = m <= n ? n : m;
  double* T1 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
  double* T2 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
  double* T3 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
  orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (m + n + 2));
  if (!T1 || !T2 || !T3 || !nodes) return ORC_ERR_NOMEM;
  orc_subproblem_tables(A, B, m, n, 0, 0, -1, g, h, T1, T2, T3, &inv);
  const char* sA = inv ? B : A;
  const char* sB = inv ? A : B;
  uint64_t len = 0;
  orc_node endn;
  /* end_type = -partial_bp[1].t = -1 (main_alignment.cpp:251) */
  int rc = orc_subproblem_traceback(sA, sB, mm, nn, 0, 0, -1, g, h, T1, T2, T3, nodes, m + n + 2,
                                    &len, &endn);
  if (score) {
    const uint64_t W = nn + 1;
    double t1 = T1[mm * W + nn], t2 = T2[mm * W + nn], t3 = T3[mm * W + nn];
    *score = dmax(dmax(t1, t2), t3);
  }
  free(T1); free(T2); free(T3);
  if (rc != ORC_OK) { free(nodes); return rc; }
  const char* hdr = "bp1\nbp1.2\nbp2\nbp3\nbp4\n";
  const uint64_t need = strlen(hdr) + 2 * (len + 1) + 1;
  if (need > cap) { free(nodes); return ORC_ERR_CAP; }
  char* l1 = (char*)malloc(len + 1);
  char* l2 = (char*)malloc(len + 1);
  orc_print_seq(A, B, m, n, nodes, len, l1, l2); /* unswapped arrays, as the reference (Q3) */
  uint64_t o = 0;
  memcpy(out + o, hdr, strlen(hdr)); o += strlen(hdr);
  memcpy(out + o, l1, len); o += len; out[o++] = '\n';
  memcpy(out + o, l2, len); o += len; out[o++] = '\n';
  out[o] = 0;
  free(l1); free(l2); free(nodes);
  return (int64_t)o;
}

/* orc_main_alignment at the reference callers' sizes (testing.cpp:261,345 pass whole
 * sequences, 13k-97k): the same single-subproblem path with integral g, h, in O(m n)
 * BYTES instead of three (m+1)(n+1) double tables.  Rows of T1/T2/T3 are int64 (the
 * reference's doubles hold exact integers here; -inf is a sentinel far below every
 * finite value, and every interior cell of start type -1 is finite, so no sum ever
 * involves it except as a losing candidate).  Each cell keeps one byte: bits 0-1 the
 * table find_alignment's T1 branch picks (the first of T1, T2, T3 at (i-1,j-1) whose
 * value equals the cell minus f, :150-155), bits 2-3 its T2 branch (:157-163), bits
 * 4-5 its T3 branch (:164-171) -- the first table in the reference's order that
 * reproduces the cell, i.e. the first maximum of the recurrence's candidates
 * (:396-398).  The walk then follows find_alignment (:105-172, quirks Q1/Q2, end rule
 * with end_type -1) and print_seq (main_alignment.cpp:32-55) over the unswapped
 * arrays.  Same output contract as orc_main_alignment. */
int64_t orc_main_alignment_dir(const char* A, const char* B, uint64_t m, uint64_t n, int64_t g, int64_t h,
                               char* out, uint64_t cap, int64_t* score) {
  const int swap = m > n;
  const char* sA = swap ? B : A;
  const char* sB = swap ? A : B;
  const uint64_t mm = swap ? n : m, nn = swap ? m : n, W = nn + 1;
  const int64_t NI = -((int64_t)1 << 50), GH = g + h;
  uint8_t* dir = (uint8_t*)malloc((mm + 1) * W);
  int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * 6 * W);
  orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (m + n + 2));
  if (!dir || !rows || !nodes) { free(dir); free(rows); free(nodes); return ORC_ERR_NOMEM; }
  int64_t *p1 = rows, *p2 = rows + W, *p3 = rows + 2 * W, *c1 = rows + 3 * W, *c2 = rows + 4 * W, *c3 = rows + 5 * W;
  /* row 0, start type -1 (compute_row(0), subproblem_alignment.cpp:212-227, :259-280) */
  p1[0] = 0; p2[0] = NI; p3[0] = NI;
  for (uint64_t j = 1; j <= nn; j++) { p1[j] = NI; p3[j] = NI; p2[j] = -h - g * (int64_t)j; }
  for (uint64_t i = 1; i <= mm; i++) {
    c1[0] = NI; c2[0] = NI; c3[0] = -h - g * (int64_t)i; /* :282-292 */
    const char a = sA[i];
    uint8_t* drow = dir + i * W;
    for (uint64_t j = 1; j <= nn; j++) {
      const int64_t f = (a == sB[j]) ? 1 : 0;
      /* T1: f + max(T1, T2, T3)(i-1, j-1); first maximum in table order */
      int64_t v1 = p1[j - 1]; unsigned k1 = 1;
      if (p2[j - 1] > v1) { v1 = p2[j - 1]; k1 = 2; }
      if (p3[j - 1] > v1) { v1 = p3[j - 1]; k1 = 3; }
      /* T2: max(T1 - g - h, T2 - g, T3 - g - h)(i, j-1) */
      int64_t v2 = c1[j - 1] - GH; unsigned k2 = 1;
      if (c2[j - 1] - g > v2) { v2 = c2[j - 1] - g; k2 = 2; }
      if (c3[j - 1] - GH > v2) { v2 = c3[j - 1] - GH; k2 = 3; }
      /* T3: max(T1 - g - h, T2 - g - h, T3 - g)(i-1, j) */
      int64_t v3 = p1[j] - GH; unsigned k3 = 1;
      if (p2[j] - GH > v3) { v3 = p2[j] - GH; k3 = 2; }
      if (p3[j] - g > v3) { v3 = p3[j] - g; k3 = 3; }
      c1[j] = f + v1;
      c2[j] = v2;
      c3[j] = v3;
      drow[j] = (uint8_t)(k1 | (k2 << 2) | (k3 << 4));
    }
    int64_t* t;
    t = p1; p1 = c1; c1 = t;
    t = p2; p2 = c2; c2 = t;
    t = p3; p3 = c3; c3 = t;
  }
  /* final cell (p* hold row mm): find_alignment's end rule with end_type -1 (:112-146) */
  const int64_t t1 = p1[nn], t2 = p2[nn], t3 = p3[nn];
  if (score) *score = t1 > t2 ? (t1 > t3 ? t1 : t3) : (t2 > t3 ? t2 : t3);
  free(rows);
  orc_node* tmp = (orc_node*)malloc(sizeof(orc_node) * (mm + nn + 2));
  if (!tmp) { free(dir); free(nodes); return ORC_ERR_NOMEM; }
  uint64_t i = mm, j = nn, cnt = 0;
  orc_node cur;
  cur.pad = 0;
  if (t1 >= t2 && t1 >= t3) { cur.t = 1; cur.i = i; cur.j = j; }
  else if (t2 >= t1 && t2 >= t3) { cur.t = 2; cur.i = 0; cur.j = j; }
  else { cur.t = 3; cur.i = i; cur.j = 0; }
  tmp[cnt++] = cur;
  int ct = cur.t;
  while (i > 0 && j > 0) {
    const unsigned d = dir[i * W + j];
    orc_node nw;
    nw.pad = 0;
    const int nt = (int)((d >> (2 * (ct - 1))) & 3u);
    nw.t = nt;
    if (ct == 1) { /* :150-156 (Q2: the T1 -> T1 node's j uses idA, 0 here) */
      nw.i = (nt == 2) ? 0 : i - 1;
      nw.j = (nt == 3) ? 0 : j - 1;
      i--; j--;
    } else if (ct == 2) { /* :157-163 */
      nw.i = (nt == 2) ? 0 : i;
      nw.j = (nt == 3) ? 0 : j - 1;
      j--;
    } else { /* :164-171 */
      nw.i = (nt == 2) ? 0 : i - 1;
      nw.j = (nt == 3) ? 0 : j;
      i--;
    }
    ct = nt;
    tmp[cnt++] = nw;
  }
  free(dir);
  const uint64_t len = cnt - 1; /* Q1: the last-created node is dropped (:170) */
  for (uint64_t k = 0; k < len; k++) nodes[k] = tmp[cnt - 2 - k];
  free(tmp);
  const char* hdr = "bp1\nbp1.2\nbp2\nbp3\nbp4\n";
  const uint64_t need = strlen(hdr) + 2 * (len + 1) + 1;
  if (need > cap) { free(nodes); return ORC_ERR_CAP; }
  uint64_t o = 0;
  memcpy(out + o, hdr, strlen(hdr)); o += strlen(hdr);
  orc_print_seq(A, B, m, n, nodes, len, out + o, out + o + len + 1); /* unswapped arrays (Q3) */
  o += len; out[o++] = '\n';
  o += len; out[o++] = '\n';
  out[o] = 0;
  free(nodes);
  return (int64_t)o;
}

/* optimal_alignment(A, B, partial_bp, m, n, p, g, h), main_alignment.cpp:202-351,
 * over the partition bp[0..nbp).  Subproblem k = Subproblem(A, B, bp[k+1].i -
 * bp[k].i, bp[k+1].j - bp[k].j, bp[k].i, bp[k].j, p', bp[k].t, -bp[k+1].t, g, h)
 * (:239-253).  Selection (:232-341): round r = 0,1,2 takes r, r+3, ... while
 * i < num-3 and then the first i past that if i < num; rounds 1-2 only run when
 * num > 3.  Stitch (:344-348): end of k-1 -> begin of k for k = 1..num-2 (the
 * last subproblem is never linked; fix_all links and solves everything).  The
 * walk from pointers[0] stops at an unsolved subproblem or an empty one
 * (alignment_begin == NULL).  Output: "bp1".."bp4" per solved subproblem, then
 * print_seq (:32-55).  *n_path receives the stitched path (path may be NULL).
 * Returns bytes of text written, or < 0. */
int64_t orc_optimal_alignment(const char* A, const char* B, uint64_t m, uint64_t n, const orc_node* bp,
                              uint64_t nbp, double g, double h, int fix_all, char* out, uint64_t cap,
                              orc_node* path, uint64_t path_cap, uint64_t* n_path) {
  if (nbp < 2) return ORC_ERR_ARG;
  const uint64_t num = nbp - 1;
  for (uint64_t k = 0; k < num; k++) {
    if (bp[k + 1].i < bp[k].i || bp[k + 1].j < bp[k].j || bp[k + 1].i > m || bp[k + 1].j > n) return ORC_ERR_ARG;
    if (bp[k + 1].i == bp[k].i && bp[k + 1].j == bp[k].j) return ORC_ERR_ARG;
  }
  char* solved = (char*)calloc(num, 1);
  uint64_t n_solved = 0;
  if (fix_all) {
    for (uint64_t k = 0; k < num; k++) solved[k] = 1;
  } else {
    const int num_sub_3 = num > 3;
    for (uint64_t r = 0; r < 3; r++) {
      if (r > 0 && !num_sub_3) break;
      uint64_t i = r;
      while (num_sub_3 && i < num - 3) { solved[i] = 1; i += 3; }
      if (i < num) solved[i] = 1;
    }
  }
  for (uint64_t k = 0; k < num; k++) n_solved += solved[k];
  orc_node* acc = (orc_node*)malloc(sizeof(orc_node) * (m + n + 2 * nbp + 2));
  uint64_t L = 0;
  const uint64_t last_link = fix_all ? num - 1 : (num >= 2 ? num - 2 : 0);
  int rc = ORC_OK;
  for (uint64_t k = 0; k < num; k++) {
    if (!solved[k]) break;
    const uint64_t lenA = bp[k + 1].i - bp[k].i, lenB = bp[k + 1].j - bp[k].j;
    const uint64_t idA = bp[k].i, idB = bp[k].j;
    const uint64_t mm = lenA <= lenB ? lenA : lenB, nn = lenA <= lenB ? lenB : lenA;
    double* T1 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
    double* T2 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
    double* T3 = (double*)malloc(sizeof(double) * (mm + 1) * (nn + 1));
    orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (lenA + lenB + 2));
    int inv;
    orc_subproblem_tables(A, B, lenA, lenB, idA, idB, bp[k].t, g, h, T1, T2, T3, &inv);
    uint64_t len = 0;
    orc_node endn;
    rc = orc_subproblem_traceback(inv ? B : A, inv ? A : B, mm, nn, inv ? idB : idA, inv ? idA : idB,
                                  -bp[k + 1].t, g, h, T1, T2, T3, nodes, lenA + lenB + 2, &len, &endn);
    free(T1); free(T2); free(T3);
    if (rc != ORC_OK) { free(nodes); break; }
    memcpy(acc + L, nodes, sizeof(orc_node) * len);
    L += len;
    free(nodes);
    if (len == 0) break;                           /* alignment_begin == NULL */
    if (k + 1 > last_link || k + 1 >= num) break;  /* end node's next stays NULL */
  }
  /* subproblems past the walk are still solved by the reference (their bp lines print) */
  free(solved);
  if (rc != ORC_OK) { free(acc); return rc; }
  if (n_path) *n_path = L;
  if (path) {
    if (L > path_cap) { free(acc); return ORC_ERR_CAP; }
    memcpy(path, acc, sizeof(orc_node) * L);
  }
  const char* hdr = "bp1\nbp1.2\nbp2\nbp3\nbp4\n";
  const uint64_t need = strlen(hdr) * n_solved + 2 * (L + 1) + 1;
  if (need > cap) { free(acc); return ORC_ERR_CAP; }
  uint64_t o = 0;
  for (uint64_t k = 0; k < n_solved; k++) { memcpy(out + o, hdr, strlen(hdr)); o += strlen(hdr); }
  char* l1 = (char*)malloc(L + 1);
  char* l2 = (char*)malloc(L + 1);
  orc_print_seq(A, B, m, n, acc, L, l1, l2);
  memcpy(out + o, l1, L); o += L; out[o++] = '\n';
  memcpy(out + o, l2, L); o += L; out[o++] = '\n';
  out[o] = 0;
  free(l1); free(l2); free(acc);
  return (int64_t)o;
}

/* ---------------------------------------------------------------------------
 * partial.cpp restated with two's-complement wrap (int32 arithmetic done in
 * uint32 so the C here has no UB).  Table shapes as the reference:
 *   T*  : (m+1) x (n+1), row stride n+1
 *   TR* : (m+2) x (n+2), row stride n+2
 * A,B are indexed A[i-1], B[j-1] (partial.cpp:105,119).
 * ------------------------------------------------------------------------- */
static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t imax3(int32_t a, int32_t b, int32_t c) {
  int32_t x = a > b ? a : b;
  return x > c ? x : c;
}

int orc_partial_tables(const char* A, const char* B, uint64_t m, uint64_t n, double g, double h,
                       int start_type, int end_type, int32_t* T1, int32_t* T2, int32_t* T3,
                       int32_t* R1, int32_t* R2, int32_t* R3) {
  const int32_t GH = (int32_t)(g + h), G = (int32_t)g;
  const uint64_t W = n + 1, WR = n + 2;
  /* initializeTables :13-31 */
  for (uint64_t k = 0; k < (m + 1) * W; k++) T1[k] = T2[k] = T3[k] = INT32_MIN;
  if (start_type == 1) T1[0] = 0;
  else if (start_type == 2) for (uint64_t j = 1; j <= n; j++) T2[j] = (int32_t)((uint32_t)(-GH) * (uint32_t)j);
  else if (start_type == 3) for (uint64_t i = 1; i <= m; i++) T3[i * W] = (int32_t)((uint32_t)(-GH) * (uint32_t)i);
  /* initializeReverseTables :33-51 */
  for (uint64_t k = 0; k < (m + 2) * WR; k++) R1[k] = R2[k] = R3[k] = INT32_MIN;
  if (end_type == 1) R1[(m + 1) * WR + n + 1] = 0;
  else if (end_type == 2) for (uint64_t j = n; j > 0; j--) R2[(m + 1) * WR + j] = (int32_t)((uint32_t)(-GH) * (uint32_t)(n - j + 1));
  else if (end_type == 3) for (uint64_t i = m; i > 0; i--) R3[i * WR + n + 1] = (int32_t)((uint32_t)(-GH) * (uint32_t)(m - i + 1));
  /* fillTablesParallel :53-65 */
  for (uint64_t i = 1; i <= m; i++)
    for (uint64_t j = 1; j <= n; j++) {
      const int32_t s = (A[i - 1] == B[j - 1]) ? 0 : 1;
      T1[i * W + j] = imax3(wadd(T1[(i - 1) * W + j - 1], s), wadd(T2[(i - 1) * W + j - 1], s),
                            wadd(T3[(i - 1) * W + j - 1], s));
      T2[i * W + j] = imax3(wsub(T1[i * W + j - 1], GH), wsub(T2[i * W + j - 1], G), wsub(T3[i * W + j - 1], GH));
      T3[i * W + j] = imax3(wsub(T1[(i - 1) * W + j], GH), wsub(T2[(i - 1) * W + j], GH), wsub(T3[(i - 1) * W + j], G));
    }
  /* fillReverseTablesParallel :67-79 */
  for (uint64_t i = m; i >= 1; i--)
    for (uint64_t j = n; j >= 1; j--) {
      const int32_t s = (A[i - 1] == B[j - 1]) ? 0 : 1;
      R1[i * WR + j] = imax3(wadd(R1[(i + 1) * WR + j + 1], s), wadd(R2[(i + 1) * WR + j + 1], s),
                             wadd(R3[(i + 1) * WR + j + 1], s));
      R2[i * WR + j] = imax3(wsub(R1[i * WR + j + 1], GH), wsub(R2[i * WR + j + 1], G), wsub(R3[i * WR + j + 1], GH));
      R3[i * WR + j] = imax3(wsub(R1[(i + 1) * WR + j], GH), wsub(R2[(i + 1) * WR + j], GH), wsub(R3[(i + 1) * WR + j], G));
    }
  return ORC_OK;
}

/* The reference sorts its partition with std::sort (partial.cpp:141-143), which is not
 * stable for more than 16 elements: points with equal (i, j) -- e.g. the (0,0,0) a band
 * with no cell above INT_MIN contributes when p > m -- come out in introsort's order.
 * This restates libstdc++'s std::sort (bits/stl_algo.h, stl_heap.h: introsort loop with
 * depth limit 2*floor(log2 n), median-of-three pivot moved to the first element,
 * unguarded Hoare partition, heapsort when the depth limit runs out, then insertion
 * sort of the first 16 and unguarded insertion of the rest) for the reference's
 * comparator (a.i < b.i || (a.i == b.i && a.j < b.j)); pinned by partial_ties.json,
 * which the reference's own build produced. */
static int orc_less(const orc_node* a, const orc_node* b) { return a->i < b->i || (a->i == b->i && a->j < b->j); }
static void orc_swap(orc_node* a, orc_node* b) { orc_node t = *a; *a = *b; *b = t; }
static void orc_push_heap(orc_node* f, long hole, long top, orc_node v) {
  long parent = (hole - 1) / 2;
  while (hole > top && orc_less(&f[parent], &v)) { f[hole] = f[parent]; hole = parent; parent = (hole - 1) / 2; }
  f[hole] = v;
}
static void orc_adjust_heap(orc_node* f, long hole, long len, orc_node v) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (orc_less(&f[second], &f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  orc_push_heap(f, hole, top, v);
}
static void orc_heap_sort(orc_node* f, long len) {
  if (len >= 2)  /* make_heap */
    for (long parent = (len - 2) / 2;; parent--) {
      orc_adjust_heap(f, parent, len, f[parent]);
      if (parent == 0) break;
    }
  for (long last = len; last > 1;) {  /* sort_heap: pop_heap */
    last--;
    const orc_node v = f[last];
    f[last] = f[0];
    orc_adjust_heap(f, 0, last, v);
  }
}
static void orc_median_to_first(orc_node* r, orc_node* a, orc_node* b, orc_node* c) {
  if (orc_less(a, b)) {
    if (orc_less(b, c)) orc_swap(r, b);
    else if (orc_less(a, c)) orc_swap(r, c);
    else orc_swap(r, a);
  } else if (orc_less(a, c)) orc_swap(r, a);
  else if (orc_less(b, c)) orc_swap(r, c);
  else orc_swap(r, b);
}
static orc_node* orc_unguarded_partition(orc_node* first, orc_node* last, const orc_node* pivot) {
  for (;;) {
    while (orc_less(first, pivot)) ++first;
    --last;
    while (orc_less(pivot, last)) --last;
    if (!(first < last)) return first;
    orc_swap(first, last);
    ++first;
  }
}
static void orc_introsort_loop(orc_node* first, orc_node* last, long depth) {
  while (last - first > 16) {
    if (depth == 0) { orc_heap_sort(first, last - first); return; }
    --depth;
    orc_node* mid = first + (last - first) / 2;
    orc_median_to_first(first, first + 1, mid, last - 1);
    orc_node* cut = orc_unguarded_partition(first + 1, last, first);
    orc_introsort_loop(cut, last, depth);
    last = cut;
  }
}
static void orc_unguarded_linear_insert(orc_node* last) {
  const orc_node v = *last;
  orc_node* next = last - 1;
  while (orc_less(&v, next)) { *last = *next; last = next; --next; }
  *last = v;
}
static void orc_insertion_sort(orc_node* first, orc_node* last) {
  if (first == last) return;
  for (orc_node* i = first + 1; i != last; ++i) {
    if (orc_less(i, first)) {
      const orc_node v = *i;
      memmove(first + 1, first, (size_t)(i - first) * sizeof(orc_node));
      *first = v;
    } else {
      orc_unguarded_linear_insert(i);
    }
  }
}
void orc_std_sort(orc_node* first, uint64_t count) {
  orc_node* last = first + count;
  if (count < 2) return;
  long lg = 0;
  for (uint64_t x = count; x > 1; x >>= 1) lg++;
  orc_introsort_loop(first, last, 2 * lg);
  if (last - first > 16) {
    orc_insertion_sort(first, first + 16);
    for (orc_node* i = first + 16; i != last; ++i) orc_unguarded_linear_insert(i);
  } else {
    orc_insertion_sort(first, last);
  }
}

/* findPartitionParallel (partial.cpp:81-146); out receives p+1 nodes sorted as the
 * reference's std::sort leaves them (orc_std_sort). */
int orc_partial_partition(const int32_t* T1, const int32_t* T2, const int32_t* T3, const int32_t* R1,
                          const int32_t* R2, const int32_t* R3, uint64_t m, uint64_t n, uint64_t p,
                          double h, orc_node* out, uint64_t cap, uint64_t* n_out) {
  if (p == 0) return ORC_ERR_ARG;
  const uint64_t W = n + 1, WR = n + 2;
  const int32_t H = (int32_t)h;
  const uint64_t bm = m / p, bn = n / p;
  uint64_t cnt = 0;
  if (cap < p + 1) return ORC_ERR_CAP;
  out[cnt].i = 0; out[cnt].j = 0; out[cnt].t = -1; out[cnt].pad = 0; cnt++;
#define VAL(i, j) imax3(wadd(T1[(i) * W + (j)], R1[(i) * WR + (j)]), \
                        wadd(wadd(T2[(i) * W + (j)], R2[(i) * WR + (j)]), H), \
                        wadd(wadd(T3[(i) * W + (j)], R3[(i) * WR + (j)]), H))
#define TYPE(i, j) ((T1[(i) * W + (j)] >= T2[(i) * W + (j)] && T1[(i) * W + (j)] >= T3[(i) * W + (j)]) ? 1 \
                    : (T2[(i) * W + (j)] >= T3[(i) * W + (j)]) ? 2 : 3)
  for (uint64_t k = 1; k < p; k++) {
    int32_t mr = INT32_MIN, mc = INT32_MIN;
    orc_node br = {0, 0, 0, 0}, bc = {0, 0, 0, 0};
    for (uint64_t i = k * bm; i < (k + 1) * bm && i <= m; i++)
      for (uint64_t j = 1; j <= n; j++) {
        const int32_t v = VAL(i, j);
        if (v > mr) { mr = v; br.i = i; br.j = j; br.t = TYPE(i, j); }
      }
    for (uint64_t j = k * bn; j < (k + 1) * bn && j <= n; j++)
      for (uint64_t i = 1; i <= m; i++) {
        const int32_t v = VAL(i, j);
        if (v > mc) { mc = v; bc.i = i; bc.j = j; bc.t = TYPE(i, j); }
      }
    out[cnt++] = (mr > mc) ? br : bc;
  }
#undef VAL
#undef TYPE
  out[cnt].i = m; out[cnt].j = n; out[cnt].t = 1; out[cnt].pad = 0; cnt++;
  orc_std_sort(out, cnt);  /* partial.cpp:141-143 */
  *n_out = cnt;
  return ORC_OK;
}

/* ---------------------------------------------------------------------------
 * Smith-Waterman local alignment (build extension; no reference equivalent).
 *   s(a,b) = a==b ? match : mismatch;  gap of length L costs open + (L-1)*extend
 *   (linear gap g  <=>  open == extend == g).
 *   E(i,j) = max(E(i,j-1) - ext, H(i,j-1) - open)    horizontal (consumes B)
 *   F(i,j) = max(F(i-1,j) - ext, H(i-1,j) - open)    vertical   (consumes A)
 *   H(i,j) = max(0, H(i-1,j-1) + s, E, F);  H(0,*) = H(*,0) = 0, E(*,0)=F(0,*)=-inf
 *   score = max H; end = first maximum in row-major order (min i, then min j).
 *   A, B are 0-based here (A[i-1] is row i).
 *   Traceback (documented tie order): in H: stop if H==0, else diag if
 *   H==Hd+s, else E if H==E, else F.  In E: open if E==H(i,j-1)-open else
 *   extend.  In F: open if F==H(i-1,j)-open else extend.
 *   cigar (optional): run-length string of M/D/I from start to end, D =
 *   horizontal move (consumes B), I = vertical move (consumes A).
 *   Hout (optional) receives H, (m+1) x (n+1) row-major.
 * ------------------------------------------------------------------------- */
int orc_sw(const char* A, const char* B, uint64_t m, uint64_t n, int32_t match, int32_t mismatch,
           int32_t open, int32_t ext, int32_t* Hout, int32_t* score, uint64_t* end_i, uint64_t* end_j,
           uint64_t* beg_i, uint64_t* beg_j, char* cigar, uint64_t cigar_cap) {
  const uint64_t W = n + 1;
  const int32_t NEG = INT32_MIN / 4;
  int32_t* H = Hout;
  int own = 0;
  const int want_tb = (cigar != NULL) || (beg_i != NULL);
  int32_t *E = NULL, *F = NULL;
  if (!H) { H = (int32_t*)malloc(sizeof(int32_t) * (m + 1) * W); own = 1; }
  if (want_tb) {
    E = (int32_t*)malloc(sizeof(int32_t) * (m + 1) * W);
    F = (int32_t*)malloc(sizeof(int32_t) * (m + 1) * W);
  }
  if (!H || (want_tb && (!E || !F))) return ORC_ERR_NOMEM;
  int32_t* Frow = (int32_t*)malloc(sizeof(int32_t) * W);
  for (uint64_t j = 0; j <= n; j++) { H[j] = 0; Frow[j] = NEG; if (want_tb) { E[j] = NEG; F[j] = NEG; } }
  int32_t best = 0;
  uint64_t bi = 0, bj = 0;
  for (uint64_t i = 1; i <= m; i++) {
    int32_t e = NEG;
    H[i * W] = 0;
    if (want_tb) { E[i * W] = NEG; F[i * W] = NEG; }
    const char a = A[i - 1];
    for (uint64_t j = 1; j <= n; j++) {
      const int32_t s = (a == B[j - 1]) ? match : mismatch;
      const int32_t el = e - ext, eo = H[i * W + j - 1] - open;
      e = el > eo ? el : eo;
      const int32_t fu = Frow[j] - ext, fo = H[(i - 1) * W + j] - open;
      const int32_t f = fu > fo ? fu : fo;
      Frow[j] = f;
      int32_t v = H[(i - 1) * W + j - 1] + s;
      if (e > v) v = e;
      if (f > v) v = f;
      if (v < 0) v = 0;
      H[i * W + j] = v;
      if (want_tb) { E[i * W + j] = e; F[i * W + j] = f; }
      if (v > best) { best = v; bi = i; bj = j; }
    }
  }
  *score = best;
  if (end_i) *end_i = bi;
  if (end_j) *end_j = bj;
  int rc = ORC_OK;
  if (want_tb) {
    /* walk back; ops collected reversed */
    char* ops = (char*)malloc(m + n + 2);
    uint64_t nops = 0, i = bi, j = bj;
    int st = 0; /* 0=H,1=E,2=F */
    if (best > 0) {
      while (1) {
        if (st == 0) {
          const int32_t v = H[i * W + j];
          if (v == 0) break;
          const int32_t s = (A[i - 1] == B[j - 1]) ? match : mismatch;
          if (v == H[(i - 1) * W + j - 1] + s) { ops[nops++] = 'M'; i--; j--; if (i == 0 || j == 0) break; }
          else if (v == E[i * W + j]) st = 1;
          else st = 2;
        } else if (st == 1) {
          const int32_t v = E[i * W + j];
          ops[nops++] = 'D';
          st = (v == H[i * W + j - 1] - open) ? 0 : 1;
          j--;
        } else {
          const int32_t v = F[i * W + j];
          ops[nops++] = 'I';
          st = (v == H[(i - 1) * W + j] - open) ? 0 : 2;
          i--;
        }
      }
    }
    if (beg_i) *beg_i = i + 1;
    if (beg_j) *beg_j = j + 1;
    if (cigar) {
      uint64_t o = 0;
      int64_t k = (int64_t)nops - 1;
      while (k >= 0) {
        char c = ops[k];
        uint64_t run = 0;
        while (k >= 0 && ops[k] == c) { run++; k--; }
        char buf[32];
        int l = 0;
        uint64_t r = run;
        char tmp[24];
        int tl = 0;
        do { tmp[tl++] = (char)('0' + r % 10); r /= 10; } while (r);
        while (tl) buf[l++] = tmp[--tl];
        buf[l++] = c;
        if (o + (uint64_t)l + 1 > cigar_cap) { rc = ORC_ERR_CAP; break; }
        memcpy(cigar + o, buf, (size_t)l);
        o += (uint64_t)l;
      }
      if (rc == ORC_OK) cigar[o] = 0;
    }
    free(ops);
    free(E); free(F);
  }
  free(Frow);
  if (own) free(H);
  return rc;
}

/* ---------------------------------------------------------------------------
 * Banded reference Gotoh (build extension for config C3): the recurrence and
 * borders of orc_subproblem_tables with start_type -1, every cell with
 * |i - j| > w treated as -inf (never computed).  Requires |m-n| <= w.
 * score = max(T1,T2,T3)[m][n].  Hout (optional, (m+1)x(n+1) row-major) gets
 * max(T1,T2,T3) as int32 for in-band interior cells and 0 elsewhere.
 * Uses O(n) memory per table row pair.
 * ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x);
uint64_t orc_mix(uint64_t i, uint64_t j);

/* digest (optional): orc_checksum_h(H, m, n, n+1, w) of the in-band H cells,
 * accumulated on the fly (C3's 97k x 97k H does not fit in host memory). */
int orc_banded_ref2(const char* A, const char* B, uint64_t m, uint64_t n, uint64_t w, double g, double h,
                    int32_t* Hout, double* score, uint64_t* digest) {
  if ((m > n ? m - n : n - m) > w) return ORC_ERR_ARG;
  const double NI = -INFINITY;
  const uint64_t W = n + 1;
  double *p1 = malloc(sizeof(double) * W), *p2 = malloc(sizeof(double) * W), *p3 = malloc(sizeof(double) * W);
  double *c1 = malloc(sizeof(double) * W), *c2 = malloc(sizeof(double) * W), *c3 = malloc(sizeof(double) * W);
  if (!p1 || !p2 || !p3 || !c1 || !c2 || !c3) return ORC_ERR_NOMEM;
  p1[0] = 0; p2[0] = NI; p3[0] = NI;
  for (uint64_t j = 1; j <= n; j++) { p1[j] = NI; p3[j] = NI; p2[j] = (j <= w) ? -h - g * (double)j : NI; }
  if (Hout) memset(Hout, 0, sizeof(int32_t) * (m + 1) * W);
  for (uint64_t j = 0; j <= n; j++) { c1[j] = NI; c2[j] = NI; c3[j] = NI; }
  uint64_t acc = 0;
  for (uint64_t i = 1; i <= m; i++) {
    /* c holds row i-2 (band [i-2-w, i-2+w]): -inf over that and row i's band and their rims */
    const uint64_t rlo = (i > w + 3) ? i - w - 3 : 0;
    const uint64_t rhi = (i + w + 1 < n) ? i + w + 1 : n;
    for (uint64_t j = rlo; j <= rhi; j++) { c1[j] = NI; c2[j] = NI; c3[j] = NI; }
    if (i <= w) c3[0] = -h - g * (double)i;
    const uint64_t jlo = (i > w) ? i - w : 1;
    const uint64_t jhi = (i + w < n) ? i + w : n;
    for (uint64_t j = jlo; j <= jhi; j++) {
      const double f = (A[i - 1] == B[j - 1]) ? 1.0 : 0.0;
      c1[j] = f + dmax(dmax(p1[j - 1], p2[j - 1]), p3[j - 1]);
      c3[j] = dmax(dmax(p1[j] - g - h, p2[j] - g - h), p3[j] - g);
      c2[j] = dmax(dmax(c1[j - 1] - g - h, c2[j - 1] - g), c3[j - 1] - g - h);
      const int32_t hv = (int32_t)dmax(dmax(c1[j], c2[j]), c3[j]);
      if (Hout) Hout[i * W + j] = hv;
      if (digest) acc += orc_mix(i, j) * (uint64_t)(uint32_t)hv;
    }
    double* t;
    t = p1; p1 = c1; c1 = t;
    t = p2; p2 = c2; c2 = t;
    t = p3; p3 = c3; c3 = t;
  }
  *score = dmax(dmax(p1[n], p2[n]), p3[n]);
  if (digest) *digest = acc;
  free(p1); free(p2); free(p3); free(c1); free(c2); free(c3);
  return ORC_OK;
}

int orc_banded_ref(const char* A, const char* B, uint64_t m, uint64_t n, uint64_t w, double g, double h,
                   int32_t* Hout, double* score) {
  return orc_banded_ref2(A, B, m, n, w, g, h, Hout, score, NULL);
}

/* ---------------------------------------------------------------------------
 * Order-independent digest of the interior of an int32 matrix: sum over
 * i in [1,m], j in [1,n] (optionally only |i-j| <= w) of
 *   mix(i,j) * (uint32)H(i,j)  mod 2^64,  mix = splitmix64(i<<32 | j) | 1.
 * The GPU computes the same digest on its own layout.
 * ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
uint64_t orc_mix(uint64_t i, uint64_t j) { return splitmix64((i << 32) | j) | 1ull; }

uint64_t orc_checksum_h(const int32_t* H, uint64_t m, uint64_t n, uint64_t stride, int64_t w) {
  uint64_t acc = 0;
  for (uint64_t i = 1; i <= m; i++)
    for (uint64_t j = 1; j <= n; j++) {
      if (w >= 0) {
        const int64_t d = (int64_t)i - (int64_t)j;
        if (d > w || -d > w) continue;
      }
      acc += orc_mix(i, j) * (uint64_t)(uint32_t)H[i * stride + j];
    }
  return acc;
}
