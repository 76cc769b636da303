/*
 * rng_stats.c — statistical check of the Tier-B counter RNG (TEST
 * INFRASTRUCTURE; tests/test_rng_stats.py runs it).
 *
 * The Tier-B stream (oracle/rtw_oracle.c tierb_state): draw k of
 * sample s of pixel p is mix(base + n * gamma) with
 * n = (p << 40) | (s << 16) | (k + 1), base = SplitMix64(seed).next().  The
 * reference renders with one sequential Xoshiro256++ stream (main.zig:300,
 * rand.zig:13-40), which no parallel renderer can reproduce, so the only
 * requirement on `mix` is that the draws a sample uses, and the draws of
 * neighbouring samples and pixels, behave as independent uniform words.  This
 * program measures exactly those relations over a block of the stream laid
 * out as a renderer uses it (NP pixels x NS samples x NK draws):
 *
 *   bits    bias of each of the 64 output bits (z-score)
 *   bytes   uniformity of each of the 8 output bytes (chi-square, 255 df)
 *   lag1    pairs (draw k, draw k+1) of one sample, each byte position
 *           against the same byte (65,535 df each; the worst of the 8 is
 *           reported) — the u,v jitter, lens-disk and unit-ball coordinates
 *           are consecutive draws (rand.zig:22-36)
 *   lag2/3  (draw k, draw k+2 / k+3), top byte x top byte
 *   hw_lag1 Hamming-weight classes of draws k and k+1 (24 df)
 *   tri     triples (k, k+1, k+2), top 5 bits each (32,767 df): the unit-ball
 *           candidate (rand.zig:24)
 *   samp    draw k of samples s and s+1 of one pixel (neighbouring counters),
 *           every byte position
 *   pix1    draw k of sample s of pixels p and p+1 (s < 4 of every pixel),
 *           every byte position
 *   pixW    pixels p and p+W, W = 1200 (the row below), top byte
 *   corr_*  Pearson correlation of the draws as Random.float-like reals for
 *           lag 1, neighbouring samples and neighbouring pixels
 *
 * Chi-square statistics are reported as z = (X - df) / sqrt(2 df); a good
 * generator gives |z| of a few units at most.  The program prints one JSON
 * object and exits 1 if any |z| exceeds the limit (default 5).
 *
 * Usage: rng_stats <mixer> <log2 pixels> <log2 samples> <log2 draws> [limit] [layout]
 *        rng_stats dump <mixer> <state>   (one output word, for cross-checks)
 * Mixers: 0 = SplitMix64 (Zig std, the round-1..4 contract), 1 = the 32-bit
 * fold form of MurmurHash3's fmix64 (x ^= x >> 32; x *= C1; ...), 2 = one
 * multiply between two folds, 3 = fold-multiply with 32-bit multipliers,
 * 4 = one fold, a 64x64 multiply, a fold and a 64x32 multiply, then a fold.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GAMMA 0x9e3779b97f4a7c15ULL

static inline uint64_t splitmix_next(uint64_t *s) {
  *s += GAMMA;
  uint64_t z = *s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

static inline uint64_t fold(uint64_t z) { return z ^ (z >> 32); }

static inline uint64_t mixer(int m, uint64_t z) {
  switch (m) {
    case 0:
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
      return z ^ (z >> 31);
    case 1:
      z = fold(z) * 0xff51afd7ed558ccdULL;
      z = fold(z) * 0xc4ceb9fe1a85ec53ULL;
      return fold(z);
    case 2:
      z = fold(z) * 0xd6e8feb86659fd93ULL;
      return fold(z);
    case 3:
      z = fold(z) * 0xed558ccdULL;
      z = fold(z) * 0x1a85ec53ULL;
      return fold(z);
    case 4:
      z = fold(z) * 0xd6e8feb86659fd93ULL;
      z = fold(z) * 0x1a85ec53ULL;
      return fold(z);
    case 5: /* Feistel half-rounds on 32-bit words: 3 */
    case 6: /* 4 */
    case 7: /* fold, then 3 */
    case 8: /* 2 */
    {
      uint32_t a = (uint32_t)(z >> 32), b = (uint32_t)z;
      const int nr = m == 5 ? 3 : m == 6 ? 4 : m == 7 ? 3 : 2;
      if (m == 7) b ^= a;
      static const uint32_t M[4] = {0xD2511F53u, 0xCD9E8D57u, 0x9E3779B1u, 0x85EBCA6Bu};
      for (int i = 0; i < nr; ++i) {
        if ((i & 1) == 0) {
          const uint64_t t = (uint64_t)b * M[i];
          a ^= (uint32_t)(t >> 32);
          b = (uint32_t)t;
        } else {
          const uint64_t t = (uint64_t)a * M[i];
          b ^= (uint32_t)(t >> 32);
          a = (uint32_t)t;
        }
      }
      return ((uint64_t)a << 32) | b;
    }
    case 9:  /* 3 half-rounds, the first multiplying the high word */
    case 10: /* 4, the first multiplying the high word */
    {
      uint32_t a = (uint32_t)(z >> 32), b = (uint32_t)z;
      const int nr = m == 9 ? 3 : 4;
      static const uint32_t M[4] = {0xD2511F53u, 0xCD9E8D57u, 0x9E3779B1u, 0x85EBCA6Bu};
      for (int i = 0; i < nr; ++i) {
        if ((i & 1) == 1) {
          const uint64_t t = (uint64_t)b * M[i];
          a ^= (uint32_t)(t >> 32);
          b = (uint32_t)t;
        } else {
          const uint64_t t = (uint64_t)a * M[i];
          b ^= (uint32_t)(t >> 32);
          a = (uint32_t)t;
        }
      }
      return ((uint64_t)a << 32) | b;
    }
    default:
      return z;
  }
}

/* Random.float(f64) without the long-leading-zero extension (a 2^-12 event
 * that does not move a correlation estimate): exponent from clz, 52-bit
 * mantissa (oracle/rtw_oracle.c ro_sm_f64). */
static inline double to_real(uint64_t v) {
  uint64_t lz = v ? (uint64_t)__builtin_clzll(v) : 64;
  if (lz > 60) lz = 60;
  const uint64_t bits = ((1022 - lz) << 52) | (v & ((1ULL << 52) - 1));
  double d;
  memcpy(&d, &bits, 8);
  return d;
}

/* Counter of the state before draw 0 of sample s of pixel p (p, s < 2^24):
 * layout 0: (p << 40) | (s << 16);  layout 1: the low bytes of p and s in bits
 * 24..31 / 16..23 (so both move the Weyl state's low word), their high 16
 * bits in bits 48..63 / 32..47. */
static inline uint64_t block_n(int layout, uint64_t p, uint64_t s) {
  if (layout == 0) return ((p << 24) | s) << 16;
  return ((p >> 8) << 48) | ((s >> 8) << 32) | ((p & 255) << 24) | ((s & 255) << 16);
}

#define C16 65536
#define C15 32768
enum { H_LAG2, H_LAG3, H_PIXW, NH };
static const char *hname[NH] = {"lag2", "lag3", "pixW"};
/* byte-wise pair tests: every byte position b of draw k against the same byte
 * of its neighbour (lag 1, next sample, next pixel) */
enum { B_LAG1, B_SAMP, B_PIX1, NB };
static const char *bname[NB] = {"lag1", "samp", "pix1"};
/* Hamming-weight classes of a 64-bit word (popcount <= 28, 29-31, 32,
 * 33-35, >= 36), for the lag-1 weight-dependency test */
static inline int hw_class(uint64_t v) {
  const int w = __builtin_popcountll(v);
  return w <= 28 ? 0 : w <= 31 ? 1 : w == 32 ? 2 : w <= 35 ? 3 : 4;
}

/* per-thread counters are u32 (a thread sees < 2^32 / 8 events per cell at
 * the sizes used); the totals are u64 */
typedef uint32_t cnt_t;
typedef struct {
  cnt_t byte[8][256];
  cnt_t pair[NH][C16];
  cnt_t bpair[NB][8][C16];
  cnt_t hw[25];
  cnt_t tri[C15];
  double sx, sxx, s1, s1n, ss, ssn, sp, spn; /* sums for the correlations */
  double n1, ns, np;
} Acc;
typedef struct {
  uint64_t byte[8][256];
  uint64_t pair[NH][C16];
  uint64_t bpair[NB][8][C16];
  uint64_t hw[25];
  uint64_t tri[C15];
  double sx, sxx, s1, s1n, ss, ssn, sp, spn; /* sums for the correlations */
  double n1, ns, np;
} Tot;

static double chi_z(const uint64_t *h, int cells) {
  double tot = 0;
  for (int i = 0; i < cells; ++i) tot += (double)h[i];
  const double e = tot / cells;
  double x = 0;
  for (int i = 0; i < cells; ++i) {
    const double d = (double)h[i] - e;
    x += d * d / e;
  }
  const double df = cells - 1;
  return (x - df) / sqrt(2 * df);
}

int main(int argc, char **argv) {
  if (argc >= 4 && !strcmp(argv[1], "dump")) {
    printf("%llu\n", (unsigned long long)mixer(atoi(argv[2]), strtoull(argv[3], 0, 0)));
    return 0;
  }
  if (argc < 5) {
    fprintf(stderr, "usage: rng_stats <mixer> <lg pixels> <lg samples> <lg draws> [limit]\n");
    return 2;
  }
  const int m = atoi(argv[1]);
  const int lp = atoi(argv[2]), ls = atoi(argv[3]), lk = atoi(argv[4]);
  const double limit = argc > 5 ? atof(argv[5]) : 5.0;
  const int layout = argc > 6 ? atoi(argv[6]) : 0;
  if (ls > 24 || lk > 16 || lp > 24) return 2;
  const uint64_t NP = 1ULL << lp, NS = 1ULL << ls, NK = 1ULL << lk;
  const uint64_t W = 1200;
  uint64_t sm = 42;
  const uint64_t base = splitmix_next(&sm);

  Tot *tot = calloc(1, sizeof(Tot));
  int nth = 1;
#ifdef _OPENMP
  nth = omp_get_max_threads();
#endif
  Acc **acc = calloc(nth, sizeof(Acc *));
  for (int t = 0; t < nth; ++t) acc[t] = calloc(1, sizeof(Acc));

#pragma omp parallel
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    Acc *A = acc[tid];
    uint64_t *cur = malloc(NK * 8), *prev = malloc(NK * 8), *nb = malloc(NK * 8);
#pragma omp for schedule(dynamic, 16)
    for (uint64_t p = 0; p < NP; ++p) {
      for (uint64_t s = 0; s < NS; ++s) {
        const uint64_t blk = base + block_n(layout, p, s) * GAMMA;
        for (uint64_t k = 0; k < NK; ++k) cur[k] = mixer(m, blk + (k + 1) * GAMMA);
        for (uint64_t k = 0; k < NK; ++k) {
          const uint64_t v = cur[k];
          for (int b = 0; b < 8; ++b) A->byte[b][(v >> (8 * b)) & 255]++;
          const double x = to_real(v);
          A->sx += x;
          A->sxx += x * x;
          if (k + 1 < NK) {
            const uint64_t w = cur[k + 1];
            for (int b = 0; b < 8; ++b) A->bpair[B_LAG1][b][(((v >> (8 * b)) & 255) << 8) | ((w >> (8 * b)) & 255)]++;
            A->hw[hw_class(v) * 5 + hw_class(w)]++;
            A->s1 += x * to_real(w);
            A->n1 += 1;
          }
          if (k + 2 < NK) {
            A->pair[H_LAG2][((v >> 56) << 8) | (cur[k + 2] >> 56)]++;
            A->tri[((v >> 59) << 10) | ((cur[k + 1] >> 59) << 5) | (cur[k + 2] >> 59)]++;
          }
          if (k + 3 < NK) A->pair[H_LAG3][((v >> 56) << 8) | (cur[k + 3] >> 56)]++;
          if (s > 0) {
            const uint64_t u = prev[k];
            for (int b = 0; b < 8; ++b) A->bpair[B_SAMP][b][(((u >> (8 * b)) & 255) << 8) | ((v >> (8 * b)) & 255)]++;
            A->ss += to_real(u) * x;
            A->ns += 1;
          }
        }
        if (s < 4) { /* neighbouring pixels: p + 1 and p + W, same sample */
          const uint64_t q[2] = {p + 1, p + W};
          for (int j = 0; j < 2; ++j) {
            const uint64_t bq = base + block_n(layout, q[j], s) * GAMMA;
            for (uint64_t k = 0; k < NK; ++k) nb[k] = mixer(m, bq + (k + 1) * GAMMA);
            for (uint64_t k = 0; k < NK; ++k) {
              if (j) {
                A->pair[H_PIXW][((cur[k] >> 56) << 8) | (nb[k] >> 56)]++;
              } else {
                for (int b = 0; b < 8; ++b)
                  A->bpair[B_PIX1][b][(((cur[k] >> (8 * b)) & 255) << 8) | ((nb[k] >> (8 * b)) & 255)]++;
                A->sp += to_real(cur[k]) * to_real(nb[k]);
                A->np += 1;
              }
            }
          }
        }
        uint64_t *t = prev;
        prev = cur;
        cur = t;
      }
    }
    free(cur);
    free(prev);
    free(nb);
  }
  for (int t = 0; t < nth; ++t) {
    Acc *A = acc[t];
    for (int b = 0; b < 8; ++b)
      for (int i = 0; i < 256; ++i) tot->byte[b][i] += A->byte[b][i];
    for (int h = 0; h < NH; ++h)
      for (int i = 0; i < C16; ++i) tot->pair[h][i] += A->pair[h][i];
    for (int i = 0; i < C15; ++i) tot->tri[i] += A->tri[i];
    for (int h = 0; h < NB; ++h)
      for (int b = 0; b < 8; ++b)
        for (int i = 0; i < C16; ++i) tot->bpair[h][b][i] += A->bpair[h][b][i];
    for (int i = 0; i < 25; ++i) tot->hw[i] += A->hw[i];
    tot->sx += A->sx;
    tot->sxx += A->sxx;
    tot->s1 += A->s1;
    tot->ss += A->ss;
    tot->sp += A->sp;
    tot->n1 += A->n1;
    tot->ns += A->ns;
    tot->np += A->np;
    free(A);
  }
  const double N = (double)(NP * NS * NK);
  double worst = 0;
  printf("{\"mixer\": %d, \"layout\": %d, \"draws\": %.0f, \"log2_draws\": %d, \"limit\": %g", m, layout, N,
         lp + ls + lk, limit);
  /* bits: z of each bit's count of ones, from the byte histograms */
  double bz = 0;
  for (int b = 0; b < 8; ++b)
    for (int i = 0; i < 8; ++i) {
      double ones = 0;
      for (int v = 0; v < 256; ++v)
        if ((v >> i) & 1) ones += (double)tot->byte[b][v];
      const double z = fabs(ones - N / 2) / sqrt(N / 4);
      if (z > bz) bz = z;
    }
  printf(", \"bits_max_z\": %.3f", bz);
  if (bz > worst) worst = bz;
  double yz = 0;
  for (int b = 0; b < 8; ++b) {
    const double z = fabs(chi_z(tot->byte[b], 256));
    if (z > yz) yz = z;
  }
  printf(", \"bytes_max_z\": %.3f", yz);
  if (yz > worst) worst = yz;
  for (int h = 0; h < NH; ++h) {
    const double z = chi_z(tot->pair[h], C16);
    printf(", \"%s_z\": %.3f", hname[h], z);
    if (fabs(z) > worst) worst = fabs(z);
  }
  for (int h = 0; h < NB; ++h) {
    double wz = 0; /* the byte position with the largest |z| */
    for (int b = 0; b < 8; ++b) {
      const double z = chi_z(tot->bpair[h][b], C16);
      if (fabs(z) > fabs(wz)) wz = z;
    }
    printf(", \"%s_bytes_max_z\": %.3f", bname[h], wz);
    if (fabs(wz) > worst) worst = fabs(wz);
  }
  { /* lag-1 Hamming-weight classes against the product of binomial(64, 1/2) */
    double pc[5] = {0, 0, 0, 0, 0}, c = 1; /* c = C(64, w) / 2^64, built up */
    for (int w = 0; w <= 64; ++w) {
      if (w > 0) c = c * (65 - w) / w;
      const double pw = c / 18446744073709551616.0;
      pc[w <= 28 ? 0 : w <= 31 ? 1 : w == 32 ? 2 : w <= 35 ? 3 : 4] += pw;
    }
    double n = 0, x = 0;
    for (int i = 0; i < 25; ++i) n += (double)tot->hw[i];
    for (int i = 0; i < 25; ++i) {
      const double e = n * pc[i / 5] * pc[i % 5], d = (double)tot->hw[i] - e;
      x += d * d / e;
    }
    const double z = (x - 24) / sqrt(48.0);
    printf(", \"hw_lag1_z\": %.3f", z);
    if (fabs(z) > worst) worst = fabs(z);
  }
  {
    const double z = chi_z(tot->tri, C15);
    printf(", \"tri_z\": %.3f", z);
    if (fabs(z) > worst) worst = fabs(z);
  }
  const double mu = tot->sx / N, var = tot->sxx / N - mu * mu;
  const double c1 = (tot->s1 / tot->n1 - mu * mu) / var;
  const double cs = (tot->ss / tot->ns - mu * mu) / var;
  const double cp = (tot->sp / tot->np - mu * mu) / var;
  /* correlation z: r * sqrt(n) */
  const double z1 = c1 * sqrt(tot->n1), zs = cs * sqrt(tot->ns), zp = cp * sqrt(tot->np);
  printf(", \"mean\": %.9f, \"corr_lag1\": %.3e, \"corr_lag1_z\": %.3f, \"corr_samp\": %.3e, \"corr_samp_z\": %.3f"
         ", \"corr_pix\": %.3e, \"corr_pix_z\": %.3f",
         mu, c1, z1, cs, zs, cp, zp);
  if (fabs(z1) > worst) worst = fabs(z1);
  if (fabs(zs) > worst) worst = fabs(zs);
  if (fabs(zp) > worst) worst = fabs(zp);
  printf(", \"worst_abs_z\": %.3f, \"pass\": %s}\n", worst, worst <= limit ? "true" : "false");
  free(tot);
  free(acc);
  return worst <= limit ? 0 : 1;
}
