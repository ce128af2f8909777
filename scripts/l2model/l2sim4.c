// LRU model of the 8 per-XCD L2s under the push's x~ gathers, with the misses split
// by source band.  Items (e0, e1, xcd) in queue order; NB persistent blocks (block b
// on XCD b % 8) take items from their XCD's queue, then steal from the next queues;
// the block with the least elapsed time advances one unit (<= UNIT entries) per step
// (time += entries + 256 per unit, + 2048 per item), as l2sim3.c.  Entries are
// sources (int32) in stream order.  Distinct lines per unit are looked up once (the
// L1/TA coalescing of a unit's gathers), in the XCD's LRU of CAP lines.
// usage: l2sim4 src.bin items.bin nv unit cap nb band_edge ...
// prints total misses and misses / distinct (unit, line) lookups per band.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
typedef struct { int32_t prev, next; uint8_t in; } node;
typedef struct { node* n; int32_t head, tail; int64_t size, cap; } lru;
static void lru_init(lru* c, int64_t nlines, int64_t cap) { c->n = calloc(nlines, sizeof(node)); c->head = c->tail = -1; c->size = 0; c->cap = cap; }
static void unlink_(lru* c, int32_t x) { node* n = c->n; if (n[x].prev >= 0) n[n[x].prev].next = n[x].next; else c->head = n[x].next; if (n[x].next >= 0) n[n[x].next].prev = n[x].prev; else c->tail = n[x].prev; }
static void push_front(lru* c, int32_t x) { node* n = c->n; n[x].prev = -1; n[x].next = c->head; if (c->head >= 0) n[c->head].prev = x; c->head = x; if (c->tail < 0) c->tail = x; }
static int access_(lru* c, int32_t x) {
  if (c->n[x].in) { unlink_(c, x); push_front(c, x); return 1; }
  if (c->size == c->cap) { int32_t t = c->tail; unlink_(c, t); c->n[t].in = 0; c->size--; }
  c->n[x].in = 1; push_front(c, x); c->size++; return 0;
}
int main(int argc, char** argv) {
  if (argc < 8) { fprintf(stderr, "usage: l2sim4 src.bin items.bin nv unit cap nb band_edge...\n"); return 2; }
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); int64_t ne = ftell(f) / 4; fseek(f, 0, SEEK_SET);
  int32_t* src = malloc(ne * 4); if (fread(src, 4, ne, f) != (size_t)ne) return 1; fclose(f);
  f = fopen(argv[2], "rb"); fseek(f, 0, SEEK_END); int64_t nt = ftell(f) / 24; fseek(f, 0, SEEK_SET);
  int64_t* T = malloc(nt * 24); if (fread(T, 24, nt, f) != (size_t)nt) return 1; fclose(f);
  int64_t nv = atoll(argv[3]), unit = atoll(argv[4]), cap = atoll(argv[5]); int nb = atoi(argv[6]);
  int nbands = argc - 7 + 1; int64_t edges[64]; edges[0] = 0;
  for (int i = 7; i < argc; ++i) edges[i - 6] = atoll(argv[i]);
  edges[nbands] = nv;
  int ls = 5; int64_t nlines = (nv >> ls) + 1;
  lru c[8]; for (int x = 0; x < 8; ++x) lru_init(&c[x], nlines, cap);
  int64_t* q[8]; int64_t qn[8] = {0}, qh[8] = {0};
  for (int x = 0; x < 8; ++x) q[x] = malloc(nt * 8);
  for (int64_t i = 0; i < nt; ++i) { int x = T[3*i+2] < 0 ? (int)(i & 7) : (int)T[3*i+2]; q[x][qn[x]++] = i; }
  int64_t *pos = calloc(nb, 8), *end = calloc(nb, 8), *t = calloc(nb, 8); int* qb = calloc(nb, 4);
  int64_t *stamp = calloc(nlines, 8), step = 0;
  int64_t miss[64] = {0}, look[64] = {0}, ent[64] = {0};
  for (int b = 0; b < nb; ++b) qb[b] = b & 7;
  #define GRAB(b) do { pos[b] = end[b] = 0; for (int k_ = 0; k_ < 8; ++k_) { int x_ = (qb[b] + k_) & 7; if (qh[x_] < qn[x_]) { int64_t i_ = q[x_][qh[x_]++]; pos[b] = T[3*i_]; end[b] = T[3*i_+1]; break; } } } while (0)
  for (int b = 0; b < nb; ++b) GRAB(b);
  while (1) {
    int bb = -1; int64_t bt = INT64_MAX;
    for (int b = 0; b < nb; ++b) if (pos[b] < end[b] && t[b] < bt) { bt = t[b]; bb = b; }
    if (bb < 0) break;
    int64_t e1 = pos[bb] + unit < end[bb] ? pos[bb] + unit : end[bb];
    ++step;
    for (int64_t e = pos[bb]; e < e1; ++e) {
      int32_t s = src[e], L = s >> ls;
      int band = 0; while (band + 1 < nbands && s >= edges[band + 1]) ++band;
      ++ent[band];
      if (stamp[L] != step) { stamp[L] = step; ++look[band]; miss[band] += !access_(&c[bb & 7], L); }
    }
    t[bb] += (e1 - pos[bb]) + 256;
    pos[bb] = e1;
    if (pos[bb] >= end[bb]) { t[bb] += 2048; GRAB(bb); }
  }
  int64_t tmax = 0, tm = 0, tl = 0; for (int b = 0; b < nb; ++b) if (t[b] > tmax) tmax = t[b];
  for (int i = 0; i < nbands; ++i) { tm += miss[i]; tl += look[i]; }
  printf("L2 misses %lld of %lld unit-line lookups; makespan %lld (ideal %lld)\n", (long long)tm, (long long)tl,
         (long long)tmax, (long long)(ne / nb));
  for (int i = 0; i < nbands; ++i)
    printf("  band [%lld, %lld): entries %.3f, lookups %lld, misses %lld (%.2f of lookups)\n", (long long)edges[i],
           (long long)edges[i + 1], (double)ent[i] / ne, (long long)look[i], (long long)miss[i],
           look[i] ? (double)miss[i] / look[i] : 0.0);
  return 0;
}
