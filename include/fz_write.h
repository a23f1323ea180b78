/* libfzwrite: the byte-exact CSV writers of the RQ drop-ins (host code, no GPU).
 *
 * The reference writes its result tables with Python's csv.writer (rq2_coverage_count.py:347-352,
 * rq2_coverage_and_added.py:221-238): str() of every cell - repr(float) for floats, str(int),
 * str(datetime), '' for None - QUOTE_MINIMAL quoting, "\r\n" line ends.  Formatting hundreds of
 * thousands (config 2) to 1e8 (config 3) cells in Python dominated the end-to-end drop-in; these
 * entry points format the same bytes natively, with worker threads over row ranges.
 *
 * Floats: repr(float) is the shortest digit string that round-trips (CPython's _Py_dg_dtoa mode
 * 0), written positionally when the decimal exponent is in [-4, 16) and as d.ddde+XX otherwise
 * (Python/pystrtod.c format_float_short with 'r' and Py_DTSF_ADD_DOT_0); the digits come from
 * C++17 std::to_chars (shortest round trip, nearest), the layout from those rules.
 * tests/test_writer.py holds every writer to the Python formatting on random and edge values and
 * on the golden outputs. */
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rows of floats (row i = vals[offs[i], offs[i+1])), comma separated, "\r\n" after each row
 * (an empty row: "\r\n") - rq2_coverage_count.py:347-352 coverage_by_session_index.csv.
 * Returns the bytes written, or -1 when cap is too small (fzw_float_rows_cap bytes always fit). */
int64_t fzw_float_rows(const double *vals, const int64_t *offs, int64_t nrows, char *out, int64_t cap, int nthreads);
int64_t fzw_float_rows_cap(const int64_t *offs, int64_t nrows);

/* The change-point rows of rq2_coverage_and_added.py:152-238 (13 cells per row; no header): per row
 * k the project id, the end / start build times (us since 1970, naive), the first / start builds'
 * modules and revisions pool ids (-1: None), the coverage rows of the two sides (-1: none -> nan),
 * diff_total (NaN or a whole number) and diff_coverage.  covered / total cells print as float when
 * the project's flag is set (pandas' upcast of a column holding NULLs), else as int; a NULL cell
 * prints nan.  row_end[k] = the byte offset after row k.  Returns the bytes written or -1. */
typedef struct {
    const int64_t *project, *t_end, *mod_f, *rev_f, *t_start, *mod_s, *rev_s, *cov_i, *cov_i1;
    const double *diff_total, *diff_coverage;
    const int64_t *c_covered, *c_total;           /* coverage table columns (by coverage row id) */
    const uint8_t *c_covered_valid, *c_total_valid;
    const uint8_t *covered_is_float, *total_is_float; /* per project */
    const char *proj_blob; const int64_t *proj_off;   /* string pools: string j = blob[off[j], off[j+1]) */
    const char *mod_blob; const int64_t *mod_off;
    const char *rev_blob; const int64_t *rev_off;
} fzw_change_cols;
int64_t fzw_change_rows(const fzw_change_cols *c, int64_t n, char *out, int64_t cap, int64_t *row_end, int nthreads);
int64_t fzw_change_rows_cap(const fzw_change_cols *c, int64_t n);

/* repr(float) of one value into out (>= 32 bytes) -> length (tests) */
int fzw_repr(double v, char *out);

#ifdef __cplusplus
}
#endif
