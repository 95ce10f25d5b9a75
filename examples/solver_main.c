/* solver_main.c -- a compiled (non-Python) host program driving libcviterbi through the C ABI
 * exactly as the Rust binding of INTEGRATION.md would: HMM::from_json (hmm.rs:242-245) ->
 * CPSolver::new (cp.rs:20) as kind "gpu-cp" -> Solver::solve -> get_objective /
 * get_solution / get_explored_nodes (main.rs:120-133) -> drop.  It stands in for the Rust
 * side, which cannot be compiled here (no Rust toolchain).
 *
 * usage: solver_main HMM_JSON INPUT [KIND]
 * INPUT (text): nseq, then nseq+1 offsets, then offsets[nseq] observations, then as many
 * components (-1 = none) and as many active flags (0/1).
 * Output: "objective <%.17g>", "explored <n>", "name <s>", then one "<seq> <state>" line per
 * element (the {prop}_0 body of main.rs:129-133). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "cviterbi.h"

static void check(cv_status st, const char* what) {
  if (st != CV_OK) {
    fprintf(stderr, "%s: %s\n", what, cv_last_error());
    exit(2);
  }
}

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(3);
  }
  return p;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s HMM_JSON INPUT [KIND]\n", argv[0]);
    return 1;
  }
  const char* kind = argc > 3 ? argv[3] : "gpu-cp";
  FILE* f = fopen(argv[2], "r");
  if (!f) {
    perror(argv[2]);
    return 1;
  }
  long long nseq = 0;
  if (fscanf(f, "%lld", &nseq) != 1 || nseq < 0) return 1;
  int64_t* off = xmalloc(sizeof(int64_t) * (size_t)(nseq + 1));
  for (long long i = 0; i <= nseq; ++i) {
    long long v;
    if (fscanf(f, "%lld", &v) != 1) return 1;
    off[i] = v;
  }
  const int64_t ne = off[nseq];
  int32_t* obs = xmalloc(sizeof(int32_t) * (size_t)ne);
  int32_t* comp = xmalloc(sizeof(int32_t) * (size_t)ne);
  uint8_t* active = xmalloc((size_t)ne);
  for (int64_t i = 0; i < ne; ++i)
    if (fscanf(f, "%d", &obs[i]) != 1) return 1;
  for (int64_t i = 0; i < ne; ++i)
    if (fscanf(f, "%d", &comp[i]) != 1) return 1;
  for (int64_t i = 0; i < ne; ++i) {
    int a;
    if (fscanf(f, "%d", &a) != 1) return 1;
    active[i] = (uint8_t)(a != 0);
  }
  fclose(f);

  cv_hmm* h = NULL;
  check(cv_hmm_from_json(argv[1], 0, &h), "cv_hmm_from_json");
  cv_superseq_desc sd = {nseq, off, obs, NULL, comp, active};
  cv_solver* s = NULL;
  check(cv_solver_create(kind, h, &sd, &s), "cv_solver_create");
  check(cv_solver_solve(s), "cv_solver_solve");
  double obj = 0.0;
  uint64_t explored = 0;
  const int32_t* sol = NULL;
  int64_t len = 0;
  check(cv_solver_get_objective(s, &obj), "cv_solver_get_objective");
  check(cv_solver_get_explored_nodes(s, &explored), "cv_solver_get_explored_nodes");
  check(cv_solver_get_solution(s, &sol, &len), "cv_solver_get_solution");
  printf("objective %.17g\nexplored %llu\nname %s\n", obj, (unsigned long long)explored, cv_solver_get_name(s));
  for (long long q = 0; q < nseq; ++q)
    for (int64_t e = off[q]; e < off[q + 1]; ++e) printf("%lld %d\n", q, sol[e]);
  cv_solver_destroy(s);
  cv_hmm_destroy(h);
  free(off);
  free(obs);
  free(comp);
  free(active);
  return 0;
}
