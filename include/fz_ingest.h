/* Native bulk ingest of the plain-format pg_dump - host C++ (no GPU):
 * libfzingest.so.  Replaces restoring data/database/backup_clean.sql into PostgreSQL (README.md:14-15)
 * and fetching the rows through program/__module/dbFile.py:16-24; feeds store.from_pg_dump.
 *
 * fz_ingest_pg_dump parses the COPY blocks of buildlog_data, total_coverage, issues and
 * project_info with `threads` worker threads into typed columns: project ids in byte order,
 * build_type / result / status codes and modules / revisions ids in first-occurrence order after
 * the schema's fixed entries (tse_amd/schema.py), timestamps as int64 microseconds of the printed
 * time (NULL = INT64_MAX), nullable numbers with validity bytes.  Cells it cannot parse are listed
 * (FZ_COL_BAD: (column code, row) pairs): the caller then falls back to its reference parser. */
#ifndef FZ_INGEST_H
#define FZ_INGEST_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct fz_ingest fz_ingest;

enum { FZ_INGEST_BUILDLOG = 0, FZ_INGEST_COVERAGE = 1, FZ_INGEST_ISSUES = 2, FZ_INGEST_PROJECT_INFO = 3,
       FZ_INGEST_HAS_NEW_ID = 16 };
/* string sets for fz_ingest_strings / fz_ingest_count: -1 projects, 0 build_type, 1 result,
 * 2 modules, 3 revisions, 4 status, -2 build names (blob + [rows + 1] offsets); -3 (count only): bad cells */
enum { FZ_COL_B_PROJECT = 0, FZ_COL_B_TYPE, FZ_COL_B_RESULT, FZ_COL_B_TIME, FZ_COL_B_MODULES, FZ_COL_B_REVISIONS,
       FZ_COL_B_NAME_NULL, FZ_COL_C_PROJECT, FZ_COL_C_DATE, FZ_COL_C_COVERAGE, FZ_COL_C_COVERAGE_OK, FZ_COL_C_COVERED,
       FZ_COL_C_COVERED_OK, FZ_COL_C_TOTAL, FZ_COL_C_TOTAL_OK, FZ_COL_I_NUMBER, FZ_COL_I_PROJECT, FZ_COL_I_RTS,
       FZ_COL_I_STATUS, FZ_COL_I_NEW_ID, FZ_COL_PI_PROJECT, FZ_COL_PI_FIRST, FZ_COL_BAD };

int fz_ingest_pg_dump(const char *path, int threads, fz_ingest **out);
const char *fz_ingest_last_error(void);
void fz_ingest_free(fz_ingest *h);
int64_t fz_ingest_rows(const fz_ingest *h, int table);
int fz_ingest_has(const fz_ingest *h, int what);
int64_t fz_ingest_count(const fz_ingest *h, int which);
/* copies a string set into blob (total bytes returned) and offsets (count + 1 entries); either may be null */
int64_t fz_ingest_strings(const fz_ingest *h, int which, char *blob, int64_t *offs);
/* copies one column (u32 projects, u8 codes / validity, i32 ids, i64 times / numbers, f64 coverage) */
int fz_ingest_column(const fz_ingest *h, int column, void *dst);

#ifdef __cplusplus
}
#endif
#endif /* FZ_INGEST_H */
