/* Cycle structure of the 180 velocity iterations (analysis tool, not product code).
 *
 * Builds the CPU oracle with a hook on every velocity iteration (HKO_VEL_HOOK), runs the bench workload
 * (strong-vs-strong, NORMAL, auto-reset, Philox streams), and for every island / TOI solve records the
 * solver state X_k (island body velocities, accumulated normal / tangent impulses) after each iteration k.
 * Reports, per solve, the iterations the kernel's period-4 exit runs and the first repeat X_k == X_j (j < k):
 * lambda = k - j is then a period of the map from j on, so X_179 == X_{k + ((179 - k) mod lambda)} and an
 * exact any-period exit could stop after k + 1 + ((179 - k) mod lambda) iterations.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/cycle_study scripts/cycle_study.c -lm && /tmp/cycle_study
 */
#define HKO_VEL_HOOK(S, Vl, nb, it, toi) cs_hook((const void *)(S), (const void *)(Vl), (nb), (it), (toi))
static void cs_hook(const void *S, const void *Vl, int nb, int it, int toi);
#define HKO_POS_HOOK(P, nb, it, toi, solved) cs_pos_hook((const void *)(P), (nb), (it), (toi), (solved))
static void cs_pos_hook(const void *P, int nb, int it, int toi, int solved);
#include <stdio.h>
#include "../oracle/hk_oracle.c"

#define MAXW 96
static __thread uint32_t g_x[VEL_ITERS][MAXW];
static __thread int g_nw;

enum { H_CUR = 0, H_EXACT = 1, H_BRENT = 2 };
static int64_t hist[2][3][VEL_ITERS + 1]; /* [toi][detector][iterations run] */
static int64_t lam_hist[2][VEL_ITERS + 1]; /* period of the solves the period-4 exit misses */
static int64_t nocyc[2], nsolve[2], slow[2];
static int64_t it_sum[2][3];
static int g_on;
static int64_t shape_hist[2][50000];
static int64_t shape_all[2][50000];

static void cs_hook(const void *Sv, const void *Vlv, int nb, int it, int toi) {
  const csolver *S = (const csolver *)Sv;
  const velv *Vl = (const velv *)Vlv;
  int n = 0;
  uint32_t *x = g_x[it];
  for (int i = 0; i < nb && n + 3 <= MAXW; ++i) {
    memcpy(&x[n++], &Vl[i].v.x, 4);
    memcpy(&x[n++], &Vl[i].v.y, 4);
    memcpy(&x[n++], &Vl[i].w, 4);
  }
  for (int i = 0; i < S->n; ++i)
    for (int j = 0; j < S->vc[i].count && n + 2 <= MAXW; ++j) {
      memcpy(&x[n++], &S->vc[i].p[j].ni, 4);
      memcpy(&x[n++], &S->vc[i].p[j].ti, 4);
    }
  g_nw = n;
  if (it != VEL_ITERS - 1 || !g_on) return;
  /* period-4 exit as the kernel runs it: compare X_k with X_{k-4} at k = 3 (mod 4), k >= 7 */
  int cur = VEL_ITERS;
  for (int k = 7; k < VEL_ITERS; k += 4)
    if (!memcmp(g_x[k], g_x[k - 4], 4 * n)) { cur = k + 1; break; }
  /* first repeat */
  int exact = VEL_ITERS, lam = 0;
  for (int k = 1; k < VEL_ITERS && !lam; ++k)
    for (int j = k - 1; j >= 0; --j)
      if (!memcmp(g_x[k], g_x[j], 4 * n)) {
        lam = k - j;
        int e = k + 1 + (VEL_ITERS - 1 - k) % lam;
        exact = e < VEL_ITERS ? e : VEL_ITERS;
        break;
      }
  /* Brent: snapshot at k = 2^i - 1, compare every later iteration until the next power */
  int brent = VEL_ITERS;
  {
    int snap = 0, pw = 1;
    for (int k = 1; k < VEL_ITERS; ++k) {
      if (!memcmp(g_x[k], g_x[snap], 4 * n)) {
        int l = k - snap, e = k + 1 + (VEL_ITERS - 1 - k) % l;
        brent = e < VEL_ITERS ? e : VEL_ITERS;
        break;
      }
      if (k == 2 * pw - 1) { snap = k; pw *= 2; }
    }
  }
  __atomic_fetch_add(&nsolve[toi], 1, __ATOMIC_RELAXED);
  {
    int sig = 0;
    for (int i = 0; i < S->n && i < 4; ++i) sig = sig * 10 + S->vc[i].count + (S->vc[i].mA != 0.0f ? 2 : 0);
    sig += 10000 * S->n;
    __atomic_fetch_add(&shape_all[toi][sig % 50000], 1, __ATOMIC_RELAXED);
  }
  __atomic_fetch_add(&hist[toi][H_CUR][cur], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&hist[toi][H_EXACT][exact], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&hist[toi][H_BRENT][brent], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&it_sum[toi][0], cur, __ATOMIC_RELAXED);
  __atomic_fetch_add(&it_sum[toi][1], exact, __ATOMIC_RELAXED);
  __atomic_fetch_add(&it_sum[toi][2], brent, __ATOMIC_RELAXED);
  if (cur == VEL_ITERS) {
    int sig = 0; /* island shape: contacts x (points, dynamic-A) */
    for (int i = 0; i < S->n && i < 4; ++i)
      sig = sig * 10 + S->vc[i].count + (S->vc[i].mA != 0.0f ? 2 : 0);
    sig += 10000 * S->n;
    __atomic_fetch_add(&shape_hist[toi][sig % 50000], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&slow[toi], 1, __ATOMIC_RELAXED);
    if (!lam) __atomic_fetch_add(&nocyc[toi], 1, __ATOMIC_RELAXED);
    else __atomic_fetch_add(&lam_hist[toi][lam], 1, __ATOMIC_RELAXED);
  }
}

/* position passes: X_k = island body positions after pass k; the loop exits when solved or after the last
 * pass.  An unsolved repeat X_k == X_j means the pass sequence is periodic from j on and never solves, so the
 * loop's result is X_{k + ((last - k) mod lambda)}. */
static __thread uint32_t g_p[POS_ITERS][MAXW];
static int64_t pos_n[2], pos_run[2], pos_exact[2], pos_full[2], pos_full_cyc[2];
static int64_t pos_hist[2][2][POS_ITERS + 1];
static void cs_pos_hook(const void *Pv, int nb, int it, int toi, int solved) {
  const posv *P = (const posv *)Pv;
  int n = 0;
  for (int i = 0; i < nb && n + 3 <= MAXW; ++i) {
    memcpy(&g_p[it][n++], &P[i].c.x, 4);
    memcpy(&g_p[it][n++], &P[i].c.y, 4);
    memcpy(&g_p[it][n++], &P[i].a, 4);
  }
  const int last = toi ? 19 : POS_ITERS - 1;
  if (!g_on || !(solved || it == last)) return;
  int exact = it + 1;
  if (!solved) {
    for (int k = 1; k <= it && exact == it + 1; ++k)
      for (int j = k - 1; j >= 0; --j)
        if (!memcmp(g_p[k], g_p[j], 4 * n)) {
          const int lam = k - j, e = k + 1 + (last - k) % lam;
          if (e < exact) exact = e;
          break;
        }
    __atomic_fetch_add(&pos_full[toi], 1, __ATOMIC_RELAXED);
    if (exact < it + 1) __atomic_fetch_add(&pos_full_cyc[toi], 1, __ATOMIC_RELAXED);
  }
  __atomic_fetch_add(&pos_n[toi], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&pos_run[toi], it + 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&pos_exact[toi], exact, __ATOMIC_RELAXED);
  __atomic_fetch_add(&pos_hist[toi][0][it + 1], 1, __ATOMIC_RELAXED);
  __atomic_fetch_add(&pos_hist[toi][1][exact], 1, __ATOMIC_RELAXED);
}

static void report_pos(int toi) {
  printf("%s position loops: %lld, passes mean %.2f (with an exact repeat exit %.2f); unsolved at the last pass: "
         "%lld, of which periodic: %lld\n", toi ? "TOI" : "island", (long long)pos_n[toi],
         (double)pos_run[toi] / pos_n[toi], (double)pos_exact[toi] / pos_n[toi], (long long)pos_full[toi],
         (long long)pos_full_cyc[toi]);
  for (int d = 0; d < 2; ++d) {
    printf("  %s passes histogram:", d ? "repeat-exit" : "as run");
    for (int k = 0; k <= POS_ITERS; ++k)
      if (pos_hist[toi][d][k]) printf(" %d:%lld", k, (long long)pos_hist[toi][d][k]);
    printf("\n");
  }
}

static void report(int toi) {
  const char *name[3] = {"period-4 (kernel)", "first repeat (exact)", "Brent"};
  printf("%s solves: %lld; period-4 exit misses %lld (%.2f%%), of which no repeat within 180: %lld\n",
         toi ? "TOI" : "island", (long long)nsolve[toi], (long long)slow[toi], 100.0 * slow[toi] / nsolve[toi],
         (long long)nocyc[toi]);
  for (int d = 0; d < 3; ++d) {
    int64_t c = 0, p50 = -1, p90 = -1, p99 = -1, p999 = -1;
    for (int k = 0; k <= VEL_ITERS; ++k) {
      c += hist[toi][d][k];
      if (p50 < 0 && c >= 0.5 * nsolve[toi]) p50 = k;
      if (p90 < 0 && c >= 0.9 * nsolve[toi]) p90 = k;
      if (p99 < 0 && c >= 0.99 * nsolve[toi]) p99 = k;
      if (p999 < 0 && c >= 0.999 * nsolve[toi]) p999 = k;
    }
    printf("  %-22s mean %.1f  p50 %lld p90 %lld p99 %lld p99.9 %lld  at 180: %.3f%%\n", name[d],
           (double)it_sum[toi][d] / nsolve[toi], (long long)p50, (long long)p90, (long long)p99, (long long)p999,
           100.0 * hist[toi][d][VEL_ITERS] / nsolve[toi]);
  }
  printf("  island shapes (contacts; per contact: points + 2 if body A dynamic) missed / all:\n");
  for (int k = 0; k < 50000; ++k)
    if (shape_hist[toi][k] * 1000 >= slow[toi])
      printf("    n=%d sig=%04d: %lld / %lld (%.2f%%)\n", k / 10000, k % 10000, (long long)shape_hist[toi][k],
             (long long)shape_all[toi][k], 100.0 * shape_hist[toi][k] / shape_all[toi][k]);
  printf("  periods of the missed solves:");
  for (int l = 1; l <= VEL_ITERS; ++l)
    if (lam_hist[toi][l]) printf(" %d:%lld", l, (long long)lam_hist[toi][l]);
  printf("\n");
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, pre = argc > 2 ? atoi(argv[2]) : 600,
            steps = argc > 3 ? atoi(argv[3]) : 200;
  const int32_t cfg[6] = {1, 0, 1, 0, 3, 3}; /* keep_mode, NORMAL, auto-reset, copy, strong, strong */
  hkov *v = hkov_create(n, cfg, 1234, 0);
  hkov_time_steps(v, pre, 0);
  memset(hist, 0, sizeof(hist));
  memset(lam_hist, 0, sizeof(lam_hist));
  memset(nocyc, 0, sizeof(nocyc));
  memset(nsolve, 0, sizeof(nsolve));
  memset(slow, 0, sizeof(slow));
  memset(it_sum, 0, sizeof(it_sum));
  g_on = 1;
  hkov_time_steps(v, steps, 0);
  printf("%d arenas, %d steps after %d\n", n, steps, pre);
  report(0);
  report(1);
  report_pos(0);
  report_pos(1);
  hkov_destroy(v);
  return 0;
}
