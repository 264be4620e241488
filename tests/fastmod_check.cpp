// Host check of kh_device.h's double-multiply remainder and quotient
// (mod_f64_32, div_f64) against the exact integer operators, at the bounds
// local_bin and SrcCommon::read_of use them under (tests/test_fastmod_cpu.py).
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../khmer_amd/csrc/kh_device.h"

using namespace kh;

static uint64_t bad = 0, checked = 0;

static void check_mod(uint64_t h, uint32_t p) {
    const uint32_t r = mod_f64_32(h, p, 1.0 / (double)p);
    checked++;
    if (r != h % p && bad++ < 10) printf("mod  h=%llu p=%u got %u want %llu\n", (unsigned long long)h, p, r,
                                         (unsigned long long)(h % p));
}
static void check_div(uint64_t x, uint64_t d) {
    const uint64_t q = div_f64(x, d, 1.0 / (double)d);
    checked++;
    if (q != x / d && bad++ < 10) printf("div  x=%llu d=%llu got %llu want %llu\n", (unsigned long long)x,
                                         (unsigned long long)d, (unsigned long long)q, (unsigned long long)(x / d));
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2000000;
    std::mt19937_64 rng(12345);
    // table sizes: the benchmark primes, small and near-2^30 sizes, powers of two
    const uint32_t ps[] = {999999937u, 999999929u, 999999893u, 999999883u, 1u, 2u, 3u, 7u, 1000003u,
                           (1u << 30) - 35u, (1u << 30) - 1u, 1u << 29, 536870909u, 100000007u};
    for (uint32_t p : ps) {
        // every hash below min(2^31 * p, 2^64): local_bin's precondition
        const double lim = std::ldexp((double)p, 31);
        const uint64_t hmax = lim >= std::ldexp(1.0, 64) ? ~0ull : (uint64_t)lim - 1;
        for (int k = 1; k <= 32; k++) {
            const uint64_t top = k == 32 ? ~0ull : (1ull << (2 * k)) - 1;
            if (top > hmax) break;
            for (uint64_t t = 0; t < n / 200; t++) check_mod(rng() & top, p);
            check_mod(top, p);
        }
        // remainders at the quotient boundaries
        for (uint64_t t = 0; t < n / 20; t++) {
            const uint64_t q = rng() % (hmax / p + 1);
            const uint64_t h = q * (uint64_t)p;
            check_mod(h, p);
            if (h) check_mod(h - 1, p);
            if (h + 1 <= hmax) check_mod(h + 1, p);
            if (h + p - 1 <= hmax) check_mod(h + p - 1, p);
        }
        check_mod(0, p);
        check_mod(hmax, p);
    }
    // read index: x < 2^52, quotient below 2^31
    const uint64_t ds[] = {1, 2, 3, 7, 11, 100, 130, 140, 1000, 12345, 1u << 20};
    for (uint64_t d : ds) {
        uint64_t xmax = ((1ull << 31) * d) - 1;
        if (xmax >= (1ull << 52)) xmax = (1ull << 52) - 1;
        for (uint64_t t = 0; t < n / 10; t++) {
            const uint64_t x = rng() % (xmax + 1);
            check_div(x, d);
            const uint64_t b = x / d * d;
            check_div(b, d);
            if (b) check_div(b - 1, d);
        }
        check_div(0, d);
        check_div(xmax, d);
    }
    printf("checked %llu, mismatches %llu\n", (unsigned long long)checked, (unsigned long long)bad);
    return bad ? 1 : 0;
}
