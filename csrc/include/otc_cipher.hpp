/*
 * otc_cipher.hpp -- C++ block-cipher interface over the gfx950 engine.
 *
 * otc::BlockCipher keeps the query/key/encrypt shape of the reference's
 * abstract interface (/root/reference/aes-gpu/Source/BlockCipher.h:48-107:
 * blockBits/blockSize/keyBits/keySize, byte2int/int2byte, makeKey(key, bits,
 * dir), encrypt/decrypt(n blocks)); otc::AesGpu implements it on one MI355X
 * (reference host class: aes-gpu/Source/AES.cu:47-282).  Differences by
 * design:
 *   - encrypt/decrypt take any buffers: device memory runs the kernels on the
 *     object's HIP stream (asynchronous; sync() waits), host memory (pageable
 *     or pinned) streams through the pinned 3-stream pipeline (synchronous);
 *   - no per-call allocation, no hidden device sync, every error throws
 *     otc::Error (the reference ignored every CUDA return code);
 *   - words are 32-bit (the reference's `uint` was 8 bytes on LP64) and
 *     byte2int/int2byte keep its big-endian GETWORD convention (AES.cu:42);
 *   - beyond ECB: ctr(), cbcDecrypt(), cbcEncryptSegments().
 * Header-only over the C API (otc.h); link with libotc.so.
 */
#ifndef OTC_CIPHER_HPP
#define OTC_CIPHER_HPP

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>

#include "otc.h"

namespace otc {

enum : unsigned { DIR_NONE = 0, DIR_ENCRYPT = 1, DIR_DECRYPT = 2, DIR_BOTH = 3 };

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char *what)
{
    if (rc != OTC_OK) throw Error(rc, std::string(what) + ": " + otc_last_error());
}

class BlockCipher {
public:
    virtual ~BlockCipher() = default;
    virtual unsigned blockBits() const = 0;
    virtual unsigned blockSize() const = 0;
    virtual unsigned keyBits() const = 0;
    virtual unsigned keySize() const = 0;
    virtual void byte2int(const uint8_t *b, uint32_t *w) const = 0;
    virtual void int2byte(const uint32_t *w, uint8_t *b) const = 0;
    virtual void makeKey(const uint8_t *cipherKey, unsigned keyBits, unsigned dir) = 0;
    virtual void encrypt(const void *pt, void *ct, size_t nblocks) = 0;
    virtual void decrypt(const void *ct, void *pt, size_t nblocks) = 0;
};

class AesGpu final : public BlockCipher {
public:
    /* stream: a hipStream_t (nullptr = default stream); impl: OTC_IMPL_* */
    explicit AesGpu(int device = 0, void *stream = nullptr, int impl = OTC_IMPL_AUTO)
        : device_(device), stream_(stream), impl_(impl)
    {
        check(otc_set_device(device), "otc_set_device");
    }

    unsigned blockBits() const override { return 128; }
    unsigned blockSize() const override { return 16; }
    unsigned keyBits() const override { return bits_; }
    unsigned keySize() const override { return bits_ / 8; }

    void byte2int(const uint8_t *b, uint32_t *w) const override
    {
        for (int i = 0; i < 4; ++i)
            w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
    }
    void int2byte(const uint32_t *w, uint8_t *b) const override
    {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) b[4 * i + j] = (uint8_t)(w[i] >> (24 - 8 * j));
    }

    void makeKey(const uint8_t *cipherKey, unsigned keyBits, unsigned dir) override
    {
        if (dir & ~(unsigned)DIR_BOTH) throw Error(OTC_ERR_ARG, "makeKey: bad direction");
        if (dir & DIR_ENCRYPT) check(otc_aes_key_init(&enc_, cipherKey, (int)keyBits, OTC_DIR_ENCRYPT), "makeKey");
        if (dir & DIR_DECRYPT) check(otc_aes_key_init(&dec_, cipherKey, (int)keyBits, OTC_DIR_DECRYPT), "makeKey");
        if (dir & DIR_ENCRYPT) has_enc_ = true;
        if (dir & DIR_DECRYPT) has_dec_ = true;
        bits_ = keyBits;
    }

    void encrypt(const void *pt, void *ct, size_t nblocks) override { ecb(pt, ct, nblocks, need(enc_, has_enc_)); }
    void decrypt(const void *ct, void *pt, size_t nblocks) override { ecb(ct, pt, nblocks, need(dec_, has_dec_)); }

    /* CTR over nbytes (any length) from the 128-bit big-endian counter
     * ctr0 + block_offset; needs the encryption schedule. */
    void ctr(const void *in, void *out, size_t nbytes, const uint8_t ctr0[16], uint64_t block_offset = 0)
    {
        const otc_aes_key &k = need(enc_, has_enc_);
        if (on_device(in, out)) {
            check(otc_aes_ctr(in, out, nbytes, &k, ctr0, block_offset, impl_, stream_), "ctr");
        } else {
            check(otc_engine_run(engine(), OTC_MODE_CTR, in, out, nbytes, &k, ctr0, block_offset, impl_, nullptr),
                  "ctr (host pipeline)");
        }
    }

    /* parallel CBC decryption (in != out); needs the decryption schedule */
    void cbcDecrypt(const void *in, void *out, size_t nbytes, const uint8_t iv[16])
    {
        const otc_aes_key &k = need(dec_, has_dec_);
        if (on_device(in, out)) {
            check(otc_aes_cbc_decrypt(in, out, nbytes, &k, iv, stream_), "cbcDecrypt");
        } else {
            check(otc_engine_run(engine(), OTC_MODE_CBC_DEC, in, out, nbytes, &k, iv, 0, impl_, nullptr),
                  "cbcDecrypt (host pipeline)");
        }
    }

    /* CBC encryption of independent seg_bytes segments, IV_s = iv0 + s
     * (device buffers) */
    void cbcEncryptSegments(const void *in, void *out, size_t seg_bytes, size_t nseg, const uint8_t iv0[16])
    {
        check(otc_aes_cbc_encrypt_segments(in, out, seg_bytes, nseg, &need(enc_, has_enc_), iv0, stream_),
              "cbcEncryptSegments");
    }

    void sync() { check(otc_device_sync(), "sync"); }
    int device() const { return device_; }

private:
    struct EngineDel {
        void operator()(otc_engine *e) const { otc_engine_destroy(e); }
    };

    static const otc_aes_key &need(const otc_aes_key &k, bool have)
    {
        if (!have) throw Error(OTC_ERR_ARG, "makeKey() was not called for this direction");
        return k;
    }
    static bool on_device(const void *a, const void *b)
    {
        const bool da = otc_ptr_kind(a) == OTC_PTR_DEVICE, db = otc_ptr_kind(b) == OTC_PTR_DEVICE;
        if (da != db) throw Error(OTC_ERR_ARG, "mixed host/device buffers");
        return da;
    }
    otc_engine *engine()
    {
        if (!eng_) {
            eng_.reset(otc_engine_create(device_, 0, 3));
            if (!eng_) throw Error(OTC_ERR_NOMEM, std::string("otc_engine_create: ") + otc_last_error());
        }
        return eng_.get();
    }
    void ecb(const void *in, void *out, size_t nblocks, const otc_aes_key &k)
    {
        if (on_device(in, out)) {
            check(otc_aes_ecb(in, out, nblocks * 16, &k, impl_, stream_), "ecb");
        } else {
            check(otc_engine_run(engine(), OTC_MODE_ECB, in, out, nblocks * 16, &k, nullptr, 0, impl_, nullptr),
                  "ecb (host pipeline)");
        }
    }

    int device_;
    void *stream_;
    int impl_;
    unsigned bits_ = 0;
    otc_aes_key enc_{}, dec_{};
    bool has_enc_ = false, has_dec_ = false;
    std::unique_ptr<otc_engine, EngineDel> eng_;
};

} // namespace otc

#endif /* OTC_CIPHER_HPP */
