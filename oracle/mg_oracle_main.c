/* mg_oracle_main.c — TEST INFRASTRUCTURE ONLY.  CLI over the C restatement,
 * output format identical to oracle/ref_harness (mode "edges"), plus "time".
 *   mg_oracle edges <fasta> <l> <out>
 *   mg_oracle time  <fasta> <l> <out>   -> JSON with hash_s / discovery_s / rows
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mg_oracle.h"

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s edges|time <fasta> <l> <out>\n", argv[0]);
    return 2;
  }
  uint64_t l = strtoull(argv[3], 0, 10);
  const char* files[1] = {argv[2]};
  mgo_dataset* ds = mgo_dataset_from_files(files, 1, l);
  if (!ds) {
    fprintf(stderr, "cannot read %s\n", argv[2]);
    return 1;
  }
  FILE* out = fopen(argv[4], "w");
  uint64_t N = mgo_num_unique(ds);
  uint64_t* super = (uint64_t*)calloc(N + 1, sizeof(uint64_t));
  mgo_row* rows = NULL;
  uint64_t nrows = 0;
  double th = 0, td = 0;
  if (mgo_overlaps(ds, l, super, &rows, &nrows, &th, &td)) return 1;
  if (!strcmp(argv[1], "time")) {
    fprintf(out, "{\"n_unique\": %llu, \"hash_s\": %.6f, \"discovery_s\": %.6f, \"directed_rows\": %llu}\n",
            (unsigned long long)N, th, td, (unsigned long long)nrows);
  } else {
    fprintf(out, "#N %llu\n", (unsigned long long)N);
    for (uint64_t i = 1; i <= N; i++) {
      fprintf(out, "#R %llu %s\n", (unsigned long long)i, mgo_read(ds, i, NULL));
      if (super[i]) fprintf(out, "#S %llu %llu\n", (unsigned long long)i, (unsigned long long)super[i]);
    }
    for (uint64_t k = 0; k < nrows; k++)
      fprintf(out, "%u %u %u %u\n", rows[k].src, rows[k].dst, (unsigned)rows[k].orient, (unsigned)rows[k].offset);
  }
  fclose(out);
  mgo_free(rows);
  free(super);
  mgo_dataset_free(ds);
  return 0;
}
