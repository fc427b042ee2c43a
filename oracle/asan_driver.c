/* Sanitizer driver for the CPU oracle (test infrastructure, tests/test_oracle_asan.py):
 * dx_oracle.c is compiled into this executable with -fsanitize=address,undefined, so the
 * whole process is instrumented without preloading anything into Python.
 *
 *   asan_driver BLOB NSTEP [NSUB]
 *
 * loads a packed model blob (dexterity_amd.blob.pack), and from qpos0 steps NSTEP control
 * steps of NSUB physics steps with a deterministic ctrl pattern, then prints the qpos sum
 * (a checksum the test compares with the uninstrumented library's). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "dx_oracle.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s BLOB NSTEP [NSUB]\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 3;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* blob = malloc((size_t)n);
  if (fread(blob, 1, (size_t)n, f) != (size_t)n) return 4;
  fclose(f);
  dxo_model* m = dxo_model_load(blob, (size_t)n);
  free(blob);
  if (!m) return 5;
  dxo_data* d = dxo_data_create(m);
  const int nstep = atoi(argv[2]), nsub = argc > 3 ? atoi(argv[3]) : 1;
  int nu = 0, nq = 0;
  double* ctrl = dxo_field(d, "ctrl", &nu);
  double* qpos = dxo_field(d, "qpos", &nq);
  int rc = 0;
  for (int s = 0; s < nstep && !rc; s++) {
    for (int i = 0; i < nu; i++) ctrl[i] = 0.5 * sin(0.7 * s + 1.3 * i);
    for (int k = 0; k < nsub && !rc; k++) rc = dxo_step(m, d);
  }
  double sum = 0;
  for (int i = 0; i < nq; i++) sum += qpos[i];
  printf("%d %.17g %d %d\n", rc, sum, dxo_ncon(d), dxo_nefc(d));
  dxo_data_free(d);
  dxo_model_free(m);
  return rc ? 6 : 0;
}
