// CPU model of k_field_wave's tiled chamfer sweeps (10x10 tiles, Jacobi across tiles, raster within): iterations to
// the fixed point from +inf and from the fixed point itself plus one ulp (the best possible upper-bound start).
//   gcc -O2 -ffp-contract=off -o /tmp/sweep_sim tools/sweep_sim.c -lm && /tmp/sweep_sim 12
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#define G 150
#define T 10
#define NT 15
static float A[G][G], B[G][G];
static int occ[G][G];
static float relax(float h, float nb, float w) { float c = nb + w; return c < h ? c : h; }
int run(int tx, int ty, int seedobst, float (*init)[G], int *front_it) {
  // init: initial values (inf or upper bound); occupied cells never change
  memcpy(A, init, sizeof(A));
  int it;
  *front_it = -1;
  for (it = 0; it < 400; ++it) {
    memcpy(B, A, sizeof(A));   // halos come from the previous iteration (B), own tile updated in place (A)
    int changed = 0;
    for (int tr = 0; tr < NT; ++tr) for (int tc = 0; tc < NT; ++tc) {
      float h[T + 2][T + 2];
      for (int i = -1; i <= T; ++i) for (int j = -1; j <= T; ++j) {
        int r = tr * T + i, c = tc * T + j;
        float v = INFINITY;
        if (r >= 0 && r < G && c >= 0 && c < G) v = (i >= 0 && i < T && j >= 0 && j < T) ? A[r][c] : B[r][c];
        if (r >= 0 && r < G && c >= 0 && c < G && occ[r][c]) v = NAN;
        h[i + 1][j + 1] = v;
      }
      for (int i = 1; i <= T; ++i) for (int j = 1; j <= T; ++j) {
        if (isnan(h[i][j])) continue;
        float m = h[i][j];
        if (!isnan(h[i-1][j-1])) m = relax(m, h[i-1][j-1], 1.414f);
        if (!isnan(h[i-1][j])) m = relax(m, h[i-1][j], 1.0f);
        if (!isnan(h[i-1][j+1])) m = relax(m, h[i-1][j+1], 1.414f);
        if (!isnan(h[i][j-1])) m = relax(m, h[i][j-1], 1.0f);
        if (m != h[i][j]) changed = 1;
        h[i][j] = m;
      }
      for (int i = T; i >= 1; --i) for (int j = T; j >= 1; --j) {
        if (isnan(h[i][j])) continue;
        float m = h[i][j];
        if (!isnan(h[i+1][j+1])) m = relax(m, h[i+1][j+1], 1.414f);
        if (!isnan(h[i+1][j])) m = relax(m, h[i+1][j], 1.0f);
        if (!isnan(h[i+1][j-1])) m = relax(m, h[i+1][j-1], 1.414f);
        if (!isnan(h[i][j+1])) m = relax(m, h[i][j+1], 1.0f);
        if (m != h[i][j]) changed = 1;
        h[i][j] = m;
      }
      for (int i = 0; i < T; ++i) for (int j = 0; j < T; ++j) if (!occ[tr*T+i][tc*T+j]) A[tr * T + i][tc * T + j] = h[i + 1][j + 1];
    }
    if (*front_it < 0) {
      int allfin = 1;
      for (int r = 1; r < G-1; ++r) for (int c = 1; c < G-1; ++c) if (!occ[r][c] && isinf(A[r][c])) allfin = 0;
      if (allfin) *front_it = it + 1;
    }
    if (!changed) break;
  }
  return it + 1;
}
int main(int argc, char **argv) {
  int trials = argc > 1 ? atoi(argv[1]) : 20;
  srand(7);
  static float init[G][G], sol[G][G];
  double s_it = 0, s_front = 0, s_ub = 0;
  for (int t = 0; t < trials; ++t) {
    memset(occ, 0, sizeof(occ));
    for (int r = 0; r < G; ++r) { occ[r][0] = occ[r][G-1] = 1; occ[0][r] = occ[G-1][r] = 1; }
    for (int o = 0; o < 16; ++o) {   // disc obstacles r = 0.5 m on a 30 m map (cell 0.2 m)
      float ox = (rand() / (float)RAND_MAX) * 24 - 12, oy = (rand() / (float)RAND_MAX) * 24 - 12;
      for (int r = 0; r < G; ++r) for (int c = 0; c < G; ++c) {
        float x = -15 + 0.2f * (c + 0.5f), y = -15 + 0.2f * (r + 0.5f);
        if (sqrtf((x-ox)*(x-ox)+(y-oy)*(y-oy)) <= 0.5f) occ[r][c] = 1;
      }
    }
    int tx = 20 + rand() % 110, ty = 20 + rand() % 110;
    occ[ty][tx] = 0;
    for (int r = 0; r < G; ++r) for (int c = 0; c < G; ++c) init[r][c] = INFINITY;
    init[ty][tx] = 0.f;
    int fr;
    int n = run(tx, ty, 0, init, &fr);
    memcpy(sol, A, sizeof(A));
    // upper bound start: the converged solution + 1 ulp-ish noise upwards (an "almost exact" bound)
    for (int r = 0; r < G; ++r) for (int c = 0; c < G; ++c) init[r][c] = (isinf(sol[r][c]) || (r==ty&&c==tx)) ? sol[r][c] : nextafterf(sol[r][c], INFINITY);
    int fr2; int n2 = run(tx, ty, 0, init, &fr2);
    // the octile bound from the straight/diagonal formula (a lower bound in exact arithmetic: not valid, just counting)
    printf("trial %d target (%d,%d): iterations %d, front complete at %d; from the solution + 1 ulp: %d\n", t, tx, ty, n, fr, n2);
    s_it += n; s_front += fr; s_ub += n2;
  }
  printf("mean iterations %.1f, front %.1f, +1ulp start %.1f\n", s_it / trials, s_front / trials, s_ub / trials);
}
