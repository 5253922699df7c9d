/* Which island shapes run a wave's velocity tail? (analysis tool, not product code; r06)
 *
 * Builds the CPU oracle with hooks on every island velocity iteration (HKO_VEL_HOOK) and on the arena being
 * stepped (HKO_ARENA_HOOK), runs the bench workload (strong-vs-strong, NORMAL, auto-reset, Philox streams), and
 * records per arena and step its island solves: contact count, the kernel's period-4 exit iteration, and the
 * island's shape (per contact: body A / body B as island-body indices, body A dynamic or static, point count).
 * It then replays the kernel's velocity-family dispatch (hk_solver.h velocity_iterations) over waves of 64
 * consecutive arenas: at every chunk start (iterations 0, 8, 16, 24, 56, 88, 120, 152) the running lanes, their
 * live contact counts and shapes, and so which family the wave runs and whether its running multi-contact lanes
 * share one shape.  Weighted by the chunk's iterations, this says how much of the velocity tail a shape-specialised
 * family (shared bodies aliased at compile time, no refresh selects) could run.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/tail_shape scripts/tail_shape_study.c -lm && /tmp/tail_shape 16384 300 60
 */
#define HKO_VEL_HOOK(S, Vl, nb, it, toi) ts_hook((const void *)(S), (const void *)(Vl), (nb), (it), (toi))
static void ts_hook(const void *S, const void *Vl, int nb, int it, int toi);
#define HKO_ARENA_HOOK(i) ts_arena(i)
#include <stdint.h>
static void ts_arena(int64_t i);
#include <stdio.h>
#include "../oracle/hk_oracle.c"

#define MAXW 96
#define MAXSOLVE 4
typedef struct {
  int n, cur;
  int iA[4], iB[4], dynA[4], cnt[4];
} solve_rec;
typedef struct {
  int ns;
  solve_rec s[MAXSOLVE];
} arena_rec;

static __thread uint32_t g_x[VEL_ITERS][MAXW];
static __thread int64_t g_arena = -1;
static arena_rec *g_rec;
static int g_on;
static int64_t toi_n[10000], toi_it[10000], toi_long[10000];

static void ts_arena(int64_t i) { g_arena = i; }

static void ts_hook(const void *Sv, const void *Vlv, int nb, int it, int toi) {
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
  if (it != VEL_ITERS - 1 || !g_on || g_arena < 0) return;
  int cur = VEL_ITERS;
  for (int k = 7; k < VEL_ITERS; k += 4)
    if (!memcmp(g_x[k], g_x[k - 4], 4 * n)) { cur = k + 1; break; }
  if (toi) { /* TOI mini-island solves: contacts x (static A?, points) and iterations run */
    int key = S->n > 3 ? 3 : S->n;
    for (int i = 0; i < S->n && i < 3; ++i) key = key * 10 + S->vc[i].count + (S->vc[i].mA != 0.0f ? 2 : 0);
    __atomic_fetch_add(&toi_n[key % 10000], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&toi_it[key % 10000], cur, __ATOMIC_RELAXED);
    if (cur >= 100) __atomic_fetch_add(&toi_long[key % 10000], 1, __ATOMIC_RELAXED);
    return;
  }
  arena_rec *r = &g_rec[g_arena];
  if (r->ns >= MAXSOLVE) return;
  solve_rec *s = &r->s[r->ns++];
  s->n = S->n;
  s->cur = cur;
  for (int i = 0; i < 4; ++i) {
    const int on = i < S->n;
    s->iA[i] = on ? S->vc[i].iA : -1;
    s->iB[i] = on ? S->vc[i].iB : -1;
    s->dynA[i] = on ? S->vc[i].mA != 0.0f : 0;
    s->cnt[i] = on ? S->vc[i].count : 0;
  }
}

/* shape key of a lane's live contacts (islands in solve order, contacts in island order): per contact
 * "A<idx|s>B<idx>p<count>", body indices renumbered in first-appearance order across the lane */
static void shape_key(const arena_rec *r, int t, char *out, int *live) {
  int map[16][8];
  for (int a = 0; a < 16; ++a)
    for (int b = 0; b < 8; ++b) map[a][b] = -1;
  int next = 0, L = 0;
  out[0] = 0;
  for (int k = 0; k < r->ns; ++k) {
    const solve_rec *s = &r->s[k];
    if (s->cur <= t) continue;
    for (int i = 0; i < s->n && i < 4; ++i) {
      int a = -1, b;
      if (s->dynA[i]) {
        if (map[k][s->iA[i]] < 0) map[k][s->iA[i]] = next++;
        a = map[k][s->iA[i]];
      }
      if (map[k][s->iB[i]] < 0) map[k][s->iB[i]] = next++;
      b = map[k][s->iB[i]];
      char buf[32];
      if (a < 0) snprintf(buf, sizeof buf, "[s%dp%d]", b, s->cnt[i]);
      else snprintf(buf, sizeof buf, "[%d%dp%d]", a, b, s->cnt[i]);
      strcat(out, buf);
      ++L;
    }
  }
  *live = L;
}

#define NKEY 4096
static char keys[NKEY][64];
static double key_w[3][NKEY];
static int nkeys;
static double gen_mix[2][2];
static double slow_tot, slow_fam[5];
static int wide_n[NKEY];
static char gen_set[2048]; /* multi-contact shapes that keep a chunk in the general family (chunks from it 8) */
static double gen_by_chunk[8]; /* lanes with >= 4 contacts live at iteration 152, by shape */
static int key_id(const char *k) {
  for (int i = 0; i < nkeys; ++i)
    if (!strcmp(keys[i], k)) return i;
  if (nkeys < NKEY) { strcpy(keys[nkeys], k); return nkeys++; }
  return NKEY - 1;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384, pre = argc > 2 ? atoi(argv[2]) : 300,
            steps = argc > 3 ? atoi(argv[3]) : 60;
  const int32_t cfg[6] = {1, 0, 1, 0, 3, 3}; /* keep_mode, NORMAL, auto-reset, copy, strong, strong */
  hkov *v = hkov_create(n, cfg, 1234, 0);
  hkov_time_steps(v, pre, 0);
  g_rec = (arena_rec *)calloc(n, sizeof(arena_rec));
  const int starts[9] = {0, 8, 16, 24, 56, 88, 120, 152, 180};
  /* per family (0 one, 1 two, 2 general): iterations x waves where the chunk's running lanes all share one
   * multi-contact shape ("uniform") or not; and the shape histogram of uniform chunks */
  double fam_it[3] = {0, 0, 0}, uni_it[3] = {0, 0, 0}, mixed_only_one[3] = {0, 0, 0};
  double tail_fam[3] = {0, 0, 0}, tail_uni[3] = {0, 0, 0};
  int64_t waves = 0;
  for (int st = 0; st < steps; ++st) {
    memset(g_rec, 0, n * sizeof(arena_rec));
    g_on = 1;
    hkov_step(v, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    g_on = 0;
    double best = -1, best_fam[5] = {0, 0, 0, 0, 0};
    char best_sig[256] = "";
    for (int w0 = 0; w0 + 64 <= n; w0 += 64) {
      ++waves;
      double wf[5] = {0, 0, 0, 0, 0};
      char wsig[256] = "";
      /* the wave's last chunk with a running lane: the chunk that ends the wave's velocity phase */
      int last_c = -1;
      for (int c = 0; c < 8; ++c)
        for (int l = 0; l < 64; ++l)
          for (int k = 0; k < g_rec[w0 + l].ns; ++k)
            if (g_rec[w0 + l].s[k].cur > starts[c]) last_c = c;
      for (int c = 0; c < 8; ++c) {
        const int t = starts[c], len = starts[c + 1] - starts[c];
        int maxlive = 0, nmulti = 0, multi_key = -1, uniform = 1, anyone = 0;
        for (int l = 0; l < 64; ++l) {
          char key[64];
          int live;
          shape_key(&g_rec[w0 + l], t, key, &live);
          if (!live) continue;
          if (live > maxlive) maxlive = live;
          if (live == 1) { anyone = 1; continue; }
          const int id = key_id(key);
          if (multi_key < 0) multi_key = id;
          else if (multi_key != id) uniform = 0;
          ++nmulti;
        }
        if (!maxlive) continue;
        const int fam = maxlive > 2 ? 2 : maxlive - 1;
        fam_it[fam] += len;
        {
          /* cost-model family: S2 / S3 when every running multi-contact lane has that shape (riders allowed) */
          const char *k = multi_key >= 0 ? keys[multi_key] : "";
          int cf;
          double cost;
          if (fam == 0) { cf = 0; cost = 86; }
          else if (fam == 1) {
            /* S2 / aliased: every multi-contact lane is S2 ([01p*][s0p*]) or TB ([*0p*][*0p*]: contact 1's B is
             * contact 0's B) */
            int all_alias = 1, all_s2 = 1;
            for (int l = 0; l < 64; ++l) {
              char key[64];
              int live;
              shape_key(&g_rec[w0 + l], t, key, &live);
              if (live != 2) continue;
              const int is_s2 = !strncmp(key, "[01p", 4) && !strncmp(key + 6, "[s0p", 4);
              const int is_tb = key[2] == '0' && key[8] == '0' && key[7] != 's' ? 1 : (key[2] == '0' && key[8] == '0');
              if (!is_s2) all_s2 = 0;
              if (!is_s2 && !is_tb) all_alias = 0;
            }
            cf = all_s2 ? 2 : all_alias ? 2 : 1;
            cost = all_s2 && uniform ? 140 : all_alias ? 180 : 225;
          } else {
            /* S3 family (r06g+): some S3 lane, every other running multi-contact lane S3 or S2 ([01p*][s0p*]) */
            int any_s3 = 0, all_ok = 1;
            for (int l = 0; l < 64; ++l) {
              char key[64];
              int live;
              shape_key(&g_rec[w0 + l], t, key, &live);
              if (live < 2) continue;
              const int is_s3 = live == 3 && !strcmp(key, "[s0p1][10p1][s1p1]");
              const int is_s2 = live == 2 && !strncmp(key, "[01p", 4) && !strncmp(key + 6, "[s0p", 4);
              any_s3 |= is_s3;
              if (!is_s3 && !is_s2) {
                all_ok = 0;
                if (c >= 1 && strlen(gen_set) + strlen(key) + 2 < sizeof gen_set && !strstr(gen_set, key)) {
                  strcat(gen_set, key);
                  strcat(gen_set, " ");
                }
              }
            }
            const int s3 = any_s3 && all_ok;
            (void)k;
            cf = s3 ? 3 : 4; cost = s3 ? 190 : 109.0 * maxlive;
            if (!s3) gen_by_chunk[c] += len;
          }
          wf[cf] += cost * len;
          if ((cf == 1 || cf == 4) && c >= 3) { /* generic two-contact or general chunk: the distinct multi-contact shapes running */
            char set[256] = "";
            for (int l = 0; l < 64; ++l) {
              char key[64];
              int live;
              shape_key(&g_rec[w0 + l], t, key, &live);
              if (live >= 2 && !strstr(set, key) && strlen(set) + strlen(key) + 2 < sizeof set) {
                strcat(set, key);
                strcat(set, " ");
              }
            }
            if (!wsig[0]) strncpy(wsig, set, sizeof wsig - 1);
          }
        }
        /* uniform: every running multi-contact lane has the same shape and no one-contact lane rides along */
        const int uni = fam == 0 || (uniform && !anyone);
        if (uni) uni_it[fam] += len;
        if (fam > 0 && uniform && anyone) mixed_only_one[fam] += len;
        if (c >= 4) {
          tail_fam[fam] += len;
          if (uni) tail_uni[fam] += len;
        }
        if (fam > 0 && uniform && multi_key >= 0 && c >= 4) key_w[anyone ? 1 : 0][multi_key] += len;
        if (c == last_c && fam > 0 && multi_key >= 0) key_w[2][multi_key] += 1;
        if (c == 7) {
          const double tot = wf[0] + wf[1] + wf[2] + wf[3] + wf[4];
          if (tot > best) { best = tot; memcpy(best_fam, wf, sizeof wf); strcpy(best_sig, wsig); }
        }
        if (fam == 2 && c >= 4) { /* general-family tail chunks: the live-contact counts of the running lanes */
          int cnt[5] = {0, 0, 0, 0, 0};
          for (int l = 0; l < 64; ++l) {
            char key[64];
            int live;
            shape_key(&g_rec[w0 + l], t, key, &live);
            if (live) ++cnt[live > 4 ? 4 : live];
          }
          gen_mix[cnt[1] > 0][cnt[2] > 0] += len;
        }
      }
    }
    for (int a = 0; a < n; ++a) { /* lanes still running at the last chunk with >= 4 live contacts: their shapes */
      char key[64];
      int live;
      shape_key(&g_rec[a], 152, key, &live);
      if (live >= 4) key_w[2][key_id(key)] += 0, wide_n[key_id(key) % NKEY] += 1;
    }
    slow_tot += best;
    printf("step %d slowest wave %.0f slots (one %.0f two-generic %.0f S2 %.0f S3 %.0f general %.0f): generic-two shapes %s\n",
           st, best, best_fam[0], best_fam[1], best_fam[2], best_fam[3], best_fam[4], best_sig);
    for (int f = 0; f < 5; ++f) slow_fam[f] += best_fam[f];
  }
  printf("%d arenas x %d steps after %d (%lld waves)\n", n, steps, pre, (long long)waves);
  printf("cost model (issue slots per iteration: one 86, two generic 225, two S2 140, S3 190, general 109 per live "
         "contact of the widest lane): slowest wave per step, mean over steps %.0f slots; its split one / two-generic "
         "/ two-S2 / S3 / general: %.0f %.0f %.0f %.0f %.0f\n", slow_tot / steps, slow_fam[0] / steps,
         slow_fam[1] / steps, slow_fam[2] / steps, slow_fam[3] / steps, slow_fam[4] / steps);
  const char *fn[3] = {"one", "two", "general"};
  for (int f = 0; f < 3; ++f)
    printf("family %-8s iterations per wave %.2f; all running multi-contact lanes one shape, no rider: %.1f%%; "
           "one shape + one-contact riders: %.1f%% | chunks from it 56: %.2f per wave, uniform %.1f%%\n",
           fn[f], fam_it[f] / waves, fam_it[f] ? 100 * uni_it[f] / fam_it[f] : 0,
           fam_it[f] ? 100 * mixed_only_one[f] / fam_it[f] : 0, tail_fam[f] / waves,
           tail_fam[f] ? 100 * tail_uni[f] / tail_fam[f] : 0);
  printf("shapes of uniform tail chunks (it >= 56), iterations per 1000 waves: [no riders] [with one-contact riders]"
         " | waves whose last chunk has this shape among its multi-contact lanes\n");
  for (int i = 0; i < nkeys; ++i)
    if (key_w[0][i] + key_w[1][i] >= 0.002 * waves || key_w[2][i] >= 0.001 * waves ||
        (strlen(keys[i]) >= 24 && key_w[2][i] >= 1))
      printf("  %-40s %9.1f %9.1f | %7.0f\n", keys[i], 1000 * key_w[0][i] / waves, 1000 * key_w[1][i] / waves,
             key_w[2][i]);
  printf("general-family tail iterations per 1000 waves by rider kinds: alone %.1f, +1-contact %.1f, +2-contact "
         "%.1f, +both %.1f\n", 1000 * gen_mix[0][0] / waves, 1000 * gen_mix[1][0] / waves, 1000 * gen_mix[0][1] / waves,
         1000 * gen_mix[1][1] / waves);
  printf("general-family chunk iterations per 1000 waves by chunk start:");
  for (int c = 0; c < 8; ++c) printf(" %d:%.1f", starts[c], 1000 * gen_by_chunk[c] / waves);
  printf("\nshapes that keep a chunk (from iteration 8) in the general family: %s\n", gen_set);
  printf("lanes with >= 4 contacts still iterating at iteration 152, by shape:\n");
  for (int i = 0; i < nkeys; ++i)
    if (wide_n[i]) printf("  %-48s %6d\n", keys[i], wide_n[i]);
  printf("TOI solves by shape (contacts, then per contact points + 2 if body A dynamic): count, mean iterations, "
         ">= 100 iterations\n");
  for (int k = 0; k < 10000; ++k)
    if (toi_n[k]) printf("  %5d %8lld %7.1f %8lld\n", k, (long long)toi_n[k], (double)toi_it[k] / toi_n[k],
                         (long long)toi_long[k]);
  hkov_destroy(v);
  return 0;
}
