/* Development: host-side parse throughput of libkhmer_hip.so's reader
 * (kh_parser_next_read in a loop: decompression + record parsing, no
 * device).  Usage: parse_bench <file> [repeats] */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include "../include/khmer_hip.h"

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s <file> [repeats]\n", argv[0]); return 2; }
    int reps = argc > 2 ? atoi(argv[2]) : 1;
    for (int r = 0; r < reps; r++) {
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        kh_parser *p = NULL;
        if (kh_parser_open(argv[1], &p) != 0) { fprintf(stderr, "open: %s\n", kh_last_error()); return 1; }
        const char *name, *seq, *qual;
        size_t nl, sl, ql;
        unsigned long long reads = 0, bases = 0;
        int rc;
        while ((rc = kh_parser_next_read(p, &name, &nl, &seq, &sl, &qual, &ql)) == 0) { reads++; bases += sl; }
        kh_parser_close(p);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
        printf("{\"file\": \"%s\", \"reads\": %llu, \"bases\": %llu, \"s\": %.3f, \"reads_per_s\": %.4g, \"rc\": %d}\n",
               argv[1], reads, bases, s, reads / s, rc);
    }
    return 0;
}
