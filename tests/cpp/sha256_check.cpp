// Host check of the SHA-256 used by the Fiat-Shamir transcript: the SHA-NI block function
// against the portable rounds on random messages and split updates, plus the FIPS 180-2
// "abc" / two-block known answers. Prints "ok" or the first mismatch.
#include <cstdio>
#include <random>
#include <vector>

#include "../../verkle-kzg_amd/csrc/host/sha256.hpp"

static bool kat(const char* msg, const char* hex) {
    vk::Sha256 h;
    uint8_t d[32];
    h.update(msg, strlen(msg));
    h.final(d);
    char got[65];
    for (int i = 0; i < 32; i++) snprintf(got + 2 * i, 3, "%02x", d[i]);
    return strcmp(got, hex) == 0;
}

int main() {
    if (!kat("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad") ||
        !kat("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
             "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1")) {
        printf("kat mismatch\n");
        return 1;
    }
    std::mt19937_64 rng(7);
    for (size_t n : {0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4096, 65537}) {
        std::vector<uint8_t> v(n);
        for (auto& x : v) x = (uint8_t)rng();
        for (size_t cut : {(size_t)0, n / 3, n / 2}) {
            vk::Sha256 a, b;
            b.portable = true;
            uint8_t da[32], db[32];
            a.update(v.data(), cut);
            a.update(v.data() + cut, n - cut);
            b.update(v.data(), n);
            a.final(da);
            b.final(db);
            if (memcmp(da, db, 32)) {
                printf("mismatch n=%zu cut=%zu\n", n, cut);
                return 1;
            }
        }
    }
    printf("ok shani=%d\n", (int)vk::sha256_have_shani());
    return 0;
}
