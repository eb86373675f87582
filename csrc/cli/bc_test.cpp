/*
 * bc_test.cpp -- exercises the C++ interface (include/otc_cipher.hpp) on one
 * GPU: FIPS-197 appendix C vectors for AES-128/192/256 through device and host
 * buffers, byte2int/int2byte (big-endian words, reference AES.cu:42), CTR and
 * CBC through both paths, and the error paths.  Prints "bc_test: OK".
 */
#include <cstdio>
#include <cstring>
#include <vector>

#include "otc_cipher.hpp"

static int fails = 0;
#define EXPECT(c)                                                        \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                     \
        }                                                                \
    } while (0)

static std::vector<uint8_t> hex(const char *s)
{
    std::vector<uint8_t> v;
    for (; s[0] && s[1]; s += 2) {
        unsigned x;
        sscanf(s, "%2x", &x);
        v.push_back((uint8_t)x);
    }
    return v;
}

int main()
{
    if (otc_device_count() < 1) {
        printf("bc_test: no GPU\n");
        return 2;
    }
    const auto pt = hex("00112233445566778899aabbccddeeff");
    const char *keys[3] = {"000102030405060708090a0b0c0d0e0f", "000102030405060708090a0b0c0d0e0f1011121314151617",
                           "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f"};
    const char *cts[3] = {"69c4e0d86a7b0430d8cdb78070b4c55a", "dda97ca4864cdfe06eaf70a0ec0d7191",
                          "8ea2b7ca516745bfeafc49904b496089"};
    try {
        otc::AesGpu aes(0);
        EXPECT(aes.blockBits() == 128 && aes.blockSize() == 16);
        uint8_t *d = (uint8_t *)otc_dev_malloc(64);
        for (int i = 0; i < 3; ++i) {
            const auto key = hex(keys[i]), ct = hex(cts[i]);
            aes.makeKey(key.data(), (unsigned)key.size() * 8, otc::DIR_BOTH);
            EXPECT(aes.keyBits() == key.size() * 8 && aes.keySize() == key.size());
            /* device path */
            uint8_t out[16];
            otc_memcpy(d, pt.data(), 16, OTC_H2D);
            aes.encrypt(d, d + 16, 1);
            aes.sync();
            otc_memcpy(out, d + 16, 16, OTC_D2H);
            EXPECT(!memcmp(out, ct.data(), 16));
            aes.decrypt(d + 16, d + 32, 1);
            aes.sync();
            otc_memcpy(out, d + 32, 16, OTC_D2H);
            EXPECT(!memcmp(out, pt.data(), 16));
            /* host path (pageable buffers through the pinned pipeline) */
            std::vector<uint8_t> h(16);
            aes.encrypt(pt.data(), h.data(), 1);
            EXPECT(!memcmp(h.data(), ct.data(), 16));
        }
        /* byte2int / int2byte: big-endian words */
        uint32_t w[4];
        aes.byte2int(pt.data(), w);
        EXPECT(w[0] == 0x00112233u && w[3] == 0xccddeeffu);
        uint8_t back[16];
        aes.int2byte(w, back);
        EXPECT(!memcmp(back, pt.data(), 16));

        /* CTR / CBC: host path == device path, odd CTR length */
        const size_t n = (1u << 20) + 5, nc = 1u << 20;
        std::vector<uint8_t> x(n), y(n), z(n);
        for (size_t i = 0; i < n; ++i) x[i] = (uint8_t)(i * 131 + 7);
        const uint8_t ctr0[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                  0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xf0};
        aes.ctr(x.data(), y.data(), n, ctr0, 3);
        uint8_t *dx = (uint8_t *)otc_dev_malloc(n + 16), *dy = (uint8_t *)otc_dev_malloc(n + 16);
        otc_memcpy(dx, x.data(), n, OTC_H2D);
        aes.ctr(dx, dy, n, ctr0, 3);
        aes.sync();
        otc_memcpy(z.data(), dy, n, OTC_D2H);
        EXPECT(y == z);
        aes.cbcDecrypt(x.data(), y.data(), nc, ctr0);
        aes.cbcDecrypt(dx, dy, nc, ctr0);
        aes.sync();
        otc_memcpy(z.data(), dy, nc, OTC_D2H);
        EXPECT(!memcmp(y.data(), z.data(), nc));

        /* errors throw */
        bool threw = false;
        try {
            otc::AesGpu fresh(0);
            fresh.encrypt(dx, dy, 1);
        } catch (const otc::Error &) {
            threw = true;
        }
        EXPECT(threw);
        threw = false;
        try {
            aes.encrypt(dx + 1, dy, 1); /* misaligned device buffer */
        } catch (const otc::Error &e) {
            threw = e.code() == OTC_ERR_ARG;
        }
        EXPECT(threw);
        otc_dev_free(d);
        otc_dev_free(dx);
        otc_dev_free(dy);
    } catch (const std::exception &e) {
        fprintf(stderr, "exception: %s\n", e.what());
        return 1;
    }
    printf(fails ? "bc_test: FAIL\n" : "bc_test: OK\n");
    return fails ? 1 : 0;
}
