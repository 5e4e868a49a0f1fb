/* sanitize_driver.c -- runs the plain-C oracle (sd_oracle_c.c, test infrastructure: the checker
 * of the GPU parity tests, never the product) under AddressSanitizer + UndefinedBehaviorSanitizer
 * on the host (sanitizers on the C restatement).
 *
 * Built as one translation unit with the oracle by tests/test_c_oracle_sanitize.py:
 *   gcc -std=gnu11 -g -O1 -fno-omit-frame-pointer -fsanitize=address,undefined
 *       -fno-sanitize-recover=all oracle/sanitize_driver.c -o oracle/_build/sdoracle_san -lm -pthread
 *
 * Input file (little endian, written by the test):
 *   int32 kind (0 MU, 1 MS, 2 MC), int32 n, int32 nbank, int32 sizeof(so_proto), int32 nthreads
 *   so_proto bank[nbank]
 *   MU/MS: int64 offsets[n+1], uint8 data[offsets[n]], uint8 npat[n], uint8 pat_id[n*10],
 *          double pat_val[n*10], uint8 ms_ok[n], int8 cp_slot[n]
 *   MC:    int64 offsets[n+1], uint8 hex[offsets[n]], int32 clock[n], int32 mcbitnum[n],
 *          uint8 mtype_lower[n], uint8 v32[n]
 * Output file: uint8 status[n], uint8 raise_kind[n], uint32 rec_begin[n], uint16 n_rec[n],
 *   uint64 rec_total, uint64 heap_total, so_res rec[rec_total], uint8 heap[heap_total]
 * Every buffer is malloc'ed at its exact size, so an out-of-bounds access is reported. */
#include "sd_oracle_c.c"

static void* rd(FILE* f, size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p || (n && fread(p, 1, n, f) != n)) {
    fprintf(stderr, "sanitize_driver: short input\n");
    exit(2);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s in out\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t* h = (int32_t*)rd(f, 5 * sizeof(int32_t));
  const int kind = h[0], n = h[1], nbank = h[2], psz = h[3], nthreads = h[4];
  if (psz != (int)sizeof(so_proto)) {
    fprintf(stderr, "sanitize_driver: so_proto size %d != %d\n", psz, (int)sizeof(so_proto));
    return 2;
  }
  so_proto* bank = (so_proto*)rd(f, (size_t)nbank * sizeof(so_proto));
  so_bank_set(bank, nbank);
  int64_t* off = (int64_t*)rd(f, (size_t)(n + 1) * sizeof(int64_t));
  uint8_t* bytes = (uint8_t*)rd(f, (size_t)off[n]);
  so_pulses pin;
  so_mcin min;
  memset(&pin, 0, sizeof pin);
  memset(&min, 0, sizeof min);
  if (kind == 2) {
    min.hex = bytes;
    min.offsets = off;
    min.clock = (int32_t*)rd(f, (size_t)n * 4);
    min.mcbitnum = (int32_t*)rd(f, (size_t)n * 4);
    min.mtype_lower = (uint8_t*)rd(f, (size_t)n);
    min.v32 = (uint8_t*)rd(f, (size_t)n);
    min.n = n;
  } else {
    pin.data = bytes;
    pin.offsets = off;
    pin.npat = (uint8_t*)rd(f, (size_t)n);
    pin.pat_id = (uint8_t*)rd(f, (size_t)n * 10);
    pin.pat_val = (double*)rd(f, (size_t)n * 10 * sizeof(double));
    pin.ms_ok = (uint8_t*)rd(f, (size_t)n);
    pin.cp_slot = (int8_t*)rd(f, (size_t)n);
    pin.n = n;
  }
  fclose(f);
  so_out o;
  memset(&o, 0, sizeof o);
  uint64_t rc = 1024, hc = 65536;
  for (;;) {
    o.status = (uint8_t*)malloc(n ? n : 1);
    o.raise_kind = (uint8_t*)malloc(n ? n : 1);
    o.rec_begin = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    o.n_rec = (uint16_t*)malloc((n ? n : 1) * sizeof(uint16_t));
    o.rec = (so_res*)malloc(rc * sizeof(so_res));
    o.heap = (uint8_t*)malloc(hc);
    o.rec_cap = rc;
    o.heap_cap = hc;
    const int r = so_demod(kind, kind == 2 ? NULL : &pin, kind == 2 ? &min : NULL, &o, nthreads);
    if (r == 0) break;
    rc = o.rec_total + 16;
    hc = o.heap_total + 16;
    free(o.status); free(o.raise_kind); free(o.rec_begin); free(o.n_rec); free(o.rec); free(o.heap);
  }
  FILE* g = fopen(argv[2], "wb");
  if (!g) return 2;
  fwrite(o.status, 1, n, g);
  fwrite(o.raise_kind, 1, n, g);
  fwrite(o.rec_begin, 4, n, g);
  fwrite(o.n_rec, 2, n, g);
  fwrite(&o.rec_total, 8, 1, g);
  fwrite(&o.heap_total, 8, 1, g);
  fwrite(o.rec, sizeof(so_res), o.rec_total, g);
  fwrite(o.heap, 1, o.heap_total, g);
  fclose(g);
  free(o.status); free(o.raise_kind); free(o.rec_begin); free(o.n_rec); free(o.rec); free(o.heap);
  free(h); free(bank); free(off); free(bytes);
  if (kind == 2) {
    free((void*)min.clock); free((void*)min.mcbitnum); free((void*)min.mtype_lower); free((void*)min.v32);
  } else {
    free((void*)pin.npat); free((void*)pin.pat_id); free((void*)pin.pat_val); free((void*)pin.ms_ok);
    free((void*)pin.cp_slot);
  }
  return 0;
}
