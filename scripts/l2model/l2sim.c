// Offline model of the PageRank push's x~ gathers through 8 per-XCD LRU L2s.
// in: src.bin (int32, entries in schedule order), tiles.bin (int64 pairs: entry
// range [e0,e1) of every tile in queue order), unit size; blocks grab tiles from
// the queue, process UNIT entries per step; time advances by entries processed.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
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
static void grab(int64_t* tiles, int64_t nt, int64_t* nxt, int b, int64_t* pos, int64_t* end) {
  int q = tiles[2] >= 0 ? (b & 7) : 8;
  while (nxt[q] < nt) {
    int64_t i = nxt[q]++;
    if (q == 8 || tiles[3*i+2] == q) { pos[b] = tiles[3*i]; end[b] = tiles[3*i+1]; return; }
  }
}
int main(int argc, char** argv) {
  if (argc < 6) { fprintf(stderr, "usage: src.bin tiles.bin nverts unit l2_lines [blocks] [line_shift]\n"); return 1; }
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); int64_t ne = ftell(f) / 4; fseek(f, 0, SEEK_SET);
  int32_t* src = malloc(ne * 4); fread(src, 4, ne, f); fclose(f);
  f = fopen(argv[2], "rb"); fseek(f, 0, SEEK_END); int64_t nt = ftell(f) / 24; fseek(f, 0, SEEK_SET);
  int64_t* tiles = malloc(nt * 24); fread(tiles, 24, nt, f); fclose(f);
  int64_t nv = atoll(argv[3]), unit = atoll(argv[4]), cap = atoll(argv[5]);
  int nb = argc > 6 ? atoi(argv[6]) : 512; int ls = argc > 7 ? atoi(argv[7]) : 5;
  int64_t nlines = (nv >> ls) + 1;
  lru c[8]; for (int x = 0; x < 8; ++x) lru_init(&c[x], nlines, cap);
  int64_t* tb = calloc(nb, 8); int64_t* pos = calloc(nb, 8); int64_t* end = calloc(nb, 8); int64_t* t = calloc(nb, 8);
  int64_t nxt[9] = {0}, miss = 0, acc = 0, uniq = 0;
#define QX(b) (tiles[2] >= 0 ? ((b) & 7) : 8)
  for (int b = 0; b < nb; ++b) { pos[b] = end[b] = 0; grab(tiles, nt, nxt, b, pos, end); }
  int64_t* stamp = calloc(nlines, 8); int64_t step = 0;
  while (1) {
    int bb = -1; int64_t bt = INT64_MAX;
    for (int b = 0; b < nb; ++b) if (pos[b] < end[b] && t[b] < bt) { bt = t[b]; bb = b; }
    if (bb < 0) break;
    int64_t e1 = pos[bb] + unit < end[bb] ? pos[bb] + unit : end[bb];
    ++step;
    for (int64_t e = pos[bb]; e < e1; ++e) {
      int32_t L = src[e] >> ls;
      if (stamp[L] != step) { stamp[L] = step; ++uniq; miss += !access_(&c[bb & 7], L); }
      ++acc;
    }
    t[bb] += (e1 - pos[bb]) + 256;  // + fixed per-unit cost
    pos[bb] = e1;
    if (pos[bb] >= end[bb]) { t[bb] += 2048; grab(tiles, nt, nxt, bb, pos, end); }
  }
  printf("entries %lld unit-distinct lines %lld (%.4f/entry) L2 misses %lld (%.4f/entry)\n", (long long)acc, (long long)uniq,
         (double)uniq / acc, (long long)miss, (double)miss / acc);
  return 0;
}
