/* Diagnostic (not product, not a test): how many distinct 128-byte lines of
 * the view do one round's applied changes touch, per delivery wave, under the
 * row-major layout (cell (node, member) at node * n + member, 16-byte cells:
 * a line holds 8 members of one node) and under a [member][node-tile of 8]
 * layout (a line holds one member of 8 consecutive nodes)?  The applied
 * (node, member) pairs come from the C oracle (oracle/sim_oracle.c, built with
 * ORC_TRACE_APPLY).  The 32-byte sector counts are the write floor of a
 * partial-line store: a dirty line is written back at sector granularity.
 *
 *   gcc -O2 -DORC_TRACE_APPLY -Ioracle tools/apply_lines.c oracle/sim_oracle.c \
 *       oracle/farmhash32.c -lm -o /tmp/apply_lines && /tmp/apply_lines 8192 40 20
 *
 * args: n rounds first_counted_round [churn_k (default n/100)] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sim_oracle.h"

#define MAXW 8
static uint64_t *pairs[MAXW];
static size_t npairs[MAXW], cap[MAXW];
static int counting;
static uint32_t N;

void orc_trace_apply(int wave, int node, int addr) {
    if (!counting) return;
    int w = wave < MAXW - 1 ? wave : MAXW - 1;
    if (npairs[w] == cap[w]) {
        cap[w] = cap[w] ? 2 * cap[w] : 1 << 16;
        pairs[w] = (uint64_t *)realloc(pairs[w], cap[w] * 8);
        if (!pairs[w]) { perror("realloc"); exit(1); }
    }
    pairs[w][npairs[w]++] = ((uint64_t)(uint32_t)node << 32) | (uint32_t)addr;
}

static int cmp64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static size_t distinct(uint64_t *k, size_t m) {
    if (!m) return 0;
    qsort(k, m, 8, cmp64);
    size_t d = 1;
    for (size_t i = 1; i < m; i++) d += k[i] != k[i - 1];
    return d;
}

int main(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s n rounds first_counted [churn_k]\n", argv[0]); return 2; }
    N = (uint32_t)atoi(argv[1]);
    int rounds = atoi(argv[2]), first = atoi(argv[3]);
    int churn = argc > 4 ? atoi(argv[4]) : (int)(N / 100);
    orc_sim *S = orc_sim_new((int)N, 1, churn, 0);
    double tot[MAXW][5] = {{0}};
    int counted = 0;
    for (int r = 0; r < rounds; r++) {
        counting = r >= first;
        for (int w = 0; w < MAXW; w++) npairs[w] = 0;
        orc_stats st;
        orc_sim_round(S, 1, &st, NULL, NULL);
        if (!counting) continue;
        counted++;
        for (int w = 0; w < MAXW; w++) {
            size_t m = npairs[w];
            if (!m) continue;
            uint64_t *k = (uint64_t *)malloc(m * 8 + 8);
            /* row-major: line = (node, member / 8); sector = (node, member / 2) */
            for (size_t i = 0; i < m; i++) k[i] = (pairs[w][i] >> 32) * (N / 8 + 1) + ((uint32_t)pairs[w][i] >> 3);
            size_t row_l = distinct(k, m);
            for (size_t i = 0; i < m; i++) k[i] = (pairs[w][i] >> 32) * (N / 2 + 1) + ((uint32_t)pairs[w][i] >> 1);
            size_t row_s = distinct(k, m);
            /* [member][node-tile of 8]: line = (member, node / 8); sector = (member, node / 2) */
            for (size_t i = 0; i < m; i++) k[i] = (uint64_t)(uint32_t)pairs[w][i] * (N / 8 + 1) + (pairs[w][i] >> 35);
            size_t til_l = distinct(k, m);
            for (size_t i = 0; i < m; i++) k[i] = (uint64_t)(uint32_t)pairs[w][i] * (N / 2 + 1) + (pairs[w][i] >> 33);
            size_t til_s = distinct(k, m);
            free(k);
            tot[w][0] += (double)m; tot[w][1] += (double)row_l; tot[w][2] += (double)til_l;
            tot[w][3] += (double)row_s; tot[w][4] += (double)til_s;
        }
    }
    printf("{\"n\": %u, \"churn_k\": %d, \"rounds_counted\": %d, \"waves\": [", N, churn, counted);
    int firstw = 1;
    for (int w = 0; w < MAXW; w++) {
        if (!tot[w][0]) continue;
        double a = tot[w][0];
        printf("%s\n  {\"wave\": %d, \"applied_per_round\": %.0f, \"row_major\": {\"lines_per_applied\": %.3f, "
               "\"sectors_per_applied\": %.3f}, \"tile8\": {\"lines_per_applied\": %.3f, \"sectors_per_applied\": %.3f}}",
               firstw ? "" : ",", w, a / counted, tot[w][1] / a, tot[w][3] / a, tot[w][2] / a, tot[w][4] / a);
        firstw = 0;
    }
    printf("\n]}\n");
    orc_sim_free(S);
    return 0;
}
