"""The device's word-based Murmur path (kh_device.h murmur_canonical_windows:
8-byte aligned window loads plus a precomputed reverse-complement stream) must
equal the byte-wise restatement of the reference's _hash_murmur
(src/oxli/kmer_hash.cc:177-198 over third-party/smhasher/MurmurHash3.cc:67-144)
for every k-mer length it takes (1..56), window alignment and byte content,
IUPAC codes and palindromes included.  Compiled for the host with g++ (the
header is shared by host and device code)."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "kh_device.h"
using namespace kh;
static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
int main() {
    const char *alpha[3] = {"ACGT", "ACGTNacgtnRYKMSWBDHVZ-", "AT"};
    static uint8_t buf[4096 + 128], rc[4096 + 128];
    long bad = 0, n = 0;
    for (int trial = 0; trial < 4000; trial++) {
        const char *a = alpha[trial % 3];
        const int na = (int)strlen(a);
        const int len = 56 + (int)(rnd() % 200);            /* one read */
        const int off = (int)(rnd() % 64);
        uint8_t *s = buf + off, *r = rc + off;
        memset(buf, 'X', sizeof buf);
        for (int i = 0; i < len; i++) s[i] = (uint8_t)a[rnd() % na];
        if (trial % 7 == 0) {                                /* a palindromic read */
            for (int i = 0; i < len / 2; i++) s[len - 1 - i] = (uint8_t)iupac_comp(s[i]);
            if (len & 1) s[len / 2] = 'A';
        }
        for (int t = 0; t < len; t++) r[t] = (uint8_t)iupac_comp(s[len - 1 - t]);   /* k_revcomp_reads */
        for (int k = 1; k <= MURMUR_WORDS_MAX; k++) {
            for (int i = 0; i + k <= len; i += 1 + (int)(rnd() % 9)) {
                const uint64_t want = murmur_canonical(s + i, k);
                const uint64_t got = murmur_canonical_windows(s + i, r + (len - k - i), k);
                n++;
                if (want != got && bad++ < 5) printf("k=%d i=%d %llx %llx\n", k, i, (unsigned long long)want,
                                                     (unsigned long long)got);
            }
        }
    }
    printf("%ld %ld\n", n, bad);
    return bad != 0;
}
'''


def test_murmur_windows_match_bytewise():
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "t.cpp")
        exe = os.path.join(tmp, "t")
        with open(src, "w") as fh:
            fh.write(PROG)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "khmer_amd", "csrc"), src, "-o",
                               exe])
        out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout[-2000:]
        n, bad = map(int, out.stdout.split()[-2:])
        assert n > 100000 and bad == 0
