// Per-XCD dynamic queues + soft lockstep gate within a round (64 consecutive items
// of an XCD queue); waiting time charged.  tiles file: int64 (e0, e1, xcd) in queue order.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
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
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); int64_t ne = ftell(f) / 4; fseek(f, 0, SEEK_SET);
  int32_t* src = malloc(ne * 4); if (fread(src, 4, ne, f) != (size_t)ne) return 1; fclose(f);
  f = fopen(argv[2], "rb"); fseek(f, 0, SEEK_END); int64_t nt = ftell(f) / 24; fseek(f, 0, SEEK_SET);
  int64_t* T = malloc(nt * 24); if (fread(T, 24, nt, f) != (size_t)nt) return 1; fclose(f);
  int64_t nv = atoll(argv[3]), unit = atoll(argv[4]), cap = atoll(argv[5]), gate = atoll(argv[6]); int R = atoi(argv[7]);
  int nb = 512, ls = 5; int64_t nlines = (nv >> ls) + 1;
  lru c[8]; for (int x = 0; x < 8; ++x) lru_init(&c[x], nlines, cap);
  int64_t* q[8]; int64_t qn[8] = {0}, qh[8] = {0};
  for (int x = 0; x < 8; ++x) q[x] = malloc(nt * 8);
  for (int64_t i = 0; i < nt; ++i) { int x = T[3*i+2] < 0 ? (int)(i & 7) : (int)T[3*i+2]; q[x][qn[x]++] = i; }
  int64_t *pos = calloc(nb, 8), *end = calloc(nb, 8), *t = calloc(nb, 8), *rnd = calloc(nb, 8);
  char* gated = calloc(nb, 1);
  int64_t *stamp = calloc(nlines, 8), step = 0, miss = 0, acc = 0, uniq = 0, idle = 0;
  #define GRAB(b) do { int x_ = (b) & 7; if (qh[x_] < qn[x_]) { int64_t k_ = qh[x_]++; int64_t i_ = q[x_][k_]; pos[b] = T[3*i_]; end[b] = T[3*i_+1]; rnd[b] = k_ / R; } else { pos[b] = end[b] = 0; } } while (0)
  for (int b = 0; b < nb; ++b) GRAB(b);
  while (1) {
    int bb = -1; int64_t bt = INT64_MAX;
    for (int b = 0; b < nb; ++b) {
      gated[b] = 0;
      if (pos[b] >= end[b]) continue;
      if (gate >= 0) {
        int64_t me = src[pos[b]], mn = INT64_MAX;
        for (int o = (b & 7); o < nb; o += 8) if (o != b && pos[o] < end[o] && rnd[o] == rnd[b] && src[pos[o]] < mn) mn = src[pos[o]];
        if (mn != INT64_MAX && me > mn + gate) { gated[b] = 1; continue; }
      }
      if (t[b] < bt) { bt = t[b]; bb = b; }
    }
    if (bb < 0) break;
    for (int b = 0; b < nb; ++b) if (gated[b] && t[b] < bt) { idle += bt - t[b]; t[b] = bt; }
    int64_t e1 = pos[bb] + unit < end[bb] ? pos[bb] + unit : end[bb];
    ++step;
    for (int64_t e = pos[bb]; e < e1; ++e) {
      int32_t L = src[e] >> ls;
      if (stamp[L] != step) { stamp[L] = step; ++uniq; miss += !access_(&c[bb & 7], L); }
      ++acc;
    }
    t[bb] += (e1 - pos[bb]) + 256;
    pos[bb] = e1;
    if (pos[bb] >= end[bb]) { t[bb] += 2048; GRAB(bb); }
  }
  int64_t tmax = 0, tsum = 0; for (int b = 0; b < nb; ++b) { if (t[b] > tmax) tmax = t[b]; tsum += t[b]; }
  printf("L2 misses %lld (%.4f/entry) makespan %lld (ideal %lld, eff %.3f) idle %.3f\n", (long long)miss,
         (double)miss / acc, (long long)tmax, (long long)((ne + 0) / nb), (double)(ne / nb) / tmax, (double)idle / tsum);
  return 0;
}
