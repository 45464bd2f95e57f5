// CPU model of k_field_wave's sweep WORK (not only its iteration count): per iteration, the tiles the kernel's
// dirty rule sweeps (a tile whose 3x3 tile neighbourhood changed in the previous iteration) and the waves that
// issue (a wave runs an iteration if any tile of its quadrant is dirty).  Same maps as tools/sweep_sim.c.
//   gcc -O2 -ffp-contract=off -o /tmp/sweep_work_sim tools/sweep_work_sim.c -lm && /tmp/sweep_work_sim 12
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#define G 150
#define T 10
#define NT 15
static float A[G][G], B[G][G];
static int occ[G][G];
static int lastc[NT + 2][NT + 2];
static int edge_mode;                 // 1: a tile is dirty if it changed, or a neighbour's cells facing it changed
static int self_c[NT + 2][NT + 2];    // per tile: changed in the previous iteration
static int face_c[NT + 2][NT + 2][9]; // per tile: its cells facing neighbour (dr, dc) changed in the previous iteration
static float relax(float h, float nb, float w) { float c = nb + w; return c < h ? c : h; }
static int quad_of(int tr, int tc) { return (tr >= 8) * 2 + (tc >= 8); }
static int ring_wave[NT][NT];   // ring mapping: wave of each tile when tiles are dealt to lanes by distance from the target
static void make_ring(int ttr, int ttc) {
  int order[NT * NT], key[NT * NT];
  for (int t = 0; t < NT * NT; ++t) {
    int tr = t / NT, tc = t % NT, dr = abs(tr - ttr), dc = abs(tc - ttc);
    key[t] = (dr > dc ? dr : dc) * 1000 + dr + dc;
    order[t] = t;
  }
  for (int i = 1; i < NT * NT; ++i) { int x = order[i], j = i; while (j > 0 && key[order[j-1]] > key[x]) { order[j] = order[j-1]; --j; } order[j] = x; }
  for (int i = 0; i < NT * NT; ++i) ring_wave[order[i] / NT][order[i] % NT] = i / 64;
}
int run(float (*init)[G], long *dirty_tiles, long *wave_its, long *hist, long *ring_its) {
  memcpy(A, init, sizeof(A));
  memset(self_c, 0, sizeof(self_c)); memset(face_c, 0, sizeof(face_c));
  for (int r = 0; r < NT + 2; ++r) for (int c = 0; c < NT + 2; ++c) lastc[r][c] = -1000;
  for (int r = 1; r <= NT; ++r) for (int c = 1; c <= NT; ++c) lastc[r][c] = 0;
  int it;
  for (it = 0; it < 400; ++it) {
    memcpy(B, A, sizeof(A));
    int changed_any = 0, nd = 0, qact[4] = {0, 0, 0, 0}, ract[4] = {0, 0, 0, 0};
    static int newc[NT][NT], nface[NT][NT][9];
    for (int tr = 0; tr < NT; ++tr) for (int tc = 0; tc < NT; ++tc) for (int f = 0; f < 9; ++f) nface[tr][tc][f] = 0;
    for (int tr = 0; tr < NT; ++tr) for (int tc = 0; tc < NT; ++tc) {
      newc[tr][tc] = 0;
      int dirty = 0;
      if (edge_mode != 1) {
        for (int dr = -1; dr <= 1; ++dr) for (int dc = -1; dc <= 1; ++dc) dirty |= lastc[tr + 1 + dr][tc + 1 + dc] >= it - 1;
      } else if (it < 2) {
        dirty = 1;
      } else {
        dirty = self_c[tr + 1][tc + 1];
        for (int dr = -1; dr <= 1; ++dr) for (int dc = -1; dc <= 1; ++dc)
          if (dr || dc) dirty |= face_c[tr + 1 + dr][tc + 1 + dc][(1 - dr) * 3 + (1 - dc)];   // neighbour's face towards us
      }
      if (!dirty) continue;
      ++nd; qact[quad_of(tr, tc)] = 1; ract[ring_wave[tr][tc]] = 1;
      float h[T + 2][T + 2];
      for (int i = -1; i <= T; ++i) for (int j = -1; j <= T; ++j) {
        int r = tr * T + i, c = tc * T + j;
        float v = INFINITY;
        if (r >= 0 && r < G && c >= 0 && c < G) v = (i >= 0 && i < T && j >= 0 && j < T) ? A[r][c] : B[r][c];
        if (r >= 0 && r < G && c >= 0 && c < G && occ[r][c]) v = NAN;
        h[i + 1][j + 1] = v;
      }
      int changed = 0;
      for (int i = 1; i <= T; ++i) for (int j = 1; j <= T; ++j) {
        if (isnan(h[i][j])) continue;
        float m = h[i][j];
        if (!isnan(h[i-1][j-1])) m = relax(m, h[i-1][j-1], 1.414f);
        if (!isnan(h[i-1][j])) m = relax(m, h[i-1][j], 1.0f);
        if (!isnan(h[i-1][j+1])) m = relax(m, h[i-1][j+1], 1.414f);
        if (!isnan(h[i][j-1])) m = relax(m, h[i][j-1], 1.0f);
        if (m != h[i][j] && (edge_mode != 2 || i == 1 || i == T || j == 1 || j == T)) changed = 1;
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
      for (int f = 0; f < 9; ++f) nface[tr][tc][f] = 0;
      for (int i = 0; i < T; ++i) for (int j = 0; j < T; ++j) {
        int r = tr * T + i, c = tc * T + j;
        if (occ[r][c]) continue;
        if (A[r][c] != h[i + 1][j + 1] && !(isinf(A[r][c]) && isinf(h[i + 1][j + 1]))) {
          // faces this cell sits on: (dr, dc) with dr = -1 if i == 0, +1 if i == T-1, dc likewise
          for (int dr = -1; dr <= 1; ++dr) for (int dc = -1; dc <= 1; ++dc) {
            if (!dr && !dc) continue;
            if (dr == -1 && i != 0) continue;
            if (dr == 1 && i != T - 1) continue;
            if (dc == -1 && j != 0) continue;
            if (dc == 1 && j != T - 1) continue;
            nface[tr][tc][(dr + 1) * 3 + (dc + 1)] = 1;
          }
        }
        A[r][c] = h[i + 1][j + 1];
      }
      newc[tr][tc] = changed;
      changed_any |= changed;
    }
    for (int tr = 0; tr < NT; ++tr) for (int tc = 0; tc < NT; ++tc) if (newc[tr][tc]) lastc[tr + 1][tc + 1] = it;
    for (int tr = 0; tr < NT; ++tr) for (int tc = 0; tc < NT; ++tc) {
      self_c[tr + 1][tc + 1] = newc[tr][tc];
      for (int f = 0; f < 9; ++f) face_c[tr + 1][tc + 1][f] = nface[tr][tc][f];
    }
    *dirty_tiles += nd;
    *wave_its += qact[0] + qact[1] + qact[2] + qact[3];
    *ring_its += ract[0] + ract[1] + ract[2] + ract[3];
    if (hist && it < 40) hist[it] += nd;
    if (!changed_any) break;
  }
  return it + 1;
}
int main(int argc, char **argv) {
  int trials = argc > 1 ? atoi(argv[1]) : 20;
  edge_mode = argc > 2 ? atoi(argv[2]) : 0;
  srand(7);
  static float init[G][G];
  long hist[40] = {0};
  double s_it = 0, s_dt = 0, s_wi = 0, s_ri = 0;
  for (int t = 0; t < trials; ++t) {
    memset(occ, 0, sizeof(occ));
    for (int r = 0; r < G; ++r) { occ[r][0] = occ[r][G-1] = 1; occ[0][r] = occ[G-1][r] = 1; }
    for (int o = 0; o < 16; ++o) {
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
    long dt = 0, wi = 0, ri = 0;
    make_ring(ty / T, tx / T);
    int n = run(init, &dt, &wi, hist, &ri);
    if (edge_mode == 2) {   // the same map with every forward cell noted: the fixed points must be the same bits
      static float ref[G][G];
      memcpy(ref, A, sizeof(A));
      long a0 = 0, b0 = 0, c0 = 0;
      edge_mode = 0;
      int n0 = run(init, &a0, &b0, NULL, &c0);
      edge_mode = 2;
      printf("  forward notes on edges only: %s, iterations %d vs %d\n",
             memcmp(ref, A, sizeof(A)) == 0 ? "same bits" : "DIFFERENT", n, n0);
    }
    printf("trial %d target (%d,%d): iterations %d, dirty tile-iterations %ld (%.1f per iteration of 225), "
           "wave-iterations %ld (lane occupancy %.2f), ring-dealt %ld\n", t, tx, ty, n, dt, (double)dt / n, wi, (double)dt / (64.0 * wi), ri);
    s_it += n; s_dt += dt; s_wi += wi; s_ri += ri;
  }
  printf("mean iterations %.1f, dirty tile-iterations %.0f, wave-iterations %.1f (quadrants) / %.1f (ring-dealt), "
         "lane occupancy %.3f\n", s_it / trials, s_dt / trials, s_wi / trials, s_ri / trials, s_dt / (64.0 * s_wi));
  printf("dirty tiles per iteration (mean over trials):");
  for (int i = 0; i < 30; ++i) printf(" %.0f", (double)hist[i] / trials);
  printf("\n");
}
