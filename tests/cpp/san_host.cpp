// san_host.cpp — host-only code of the product under ASan + UBSan
// (oncrpc4j_amd/csrc/Makefile `sanitize`, run by tests/test_sanitize.py, no
// GPU): the C-ABI's schema compiler and argument validation
// (xdrg_abi.cpp) over random and malformed field tapes, and the C++
// mirror's XdrBuffer growth (Xdr.java:1020-1026,
// GrizzlyMemoryManager.java:46-53).  Exit 0 = every check held.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "xdrg.h"
#include "xdrg_host.hpp"

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

using oncrpc4j::xdr::XdrBuffer;

static void schemas(std::mt19937_64 &rng) {
    for (int r = 0; r < 4000; ++r) {
        const size_t nf = rng() % 40;   // beyond the field limit too
        std::vector<xdrg_field> f(nf ? nf : 1);
        for (auto &x : f) {
            x.type = (uint32_t)(rng() % 14);          // includes invalid 0 and 13
            x.kind = (uint32_t)(rng() % 4);           // includes invalid 3
            x.count = (uint32_t)(rng() % 3 ? rng() % 70 : rng());
            x.reserved = rng() % 50 == 0;
        }
        std::vector<xdrg_cond> c(rng() % 4);
        std::vector<int32_t> vals(8);
        for (auto &v : vals) v = (int32_t)rng();
        for (auto &x : c) {
            x.field = (uint32_t)(rng() % (nf + 2));
            x.disc = (uint32_t)(rng() % (nf + 2));
            x.negate = (uint32_t)(rng() % 3);
            x.nvalues = (uint32_t)(rng() % 9);
            x.values = rng() % 10 ? vals.data() : nullptr;
        }
        xdrg_schema *s = nullptr;
        const int st = c.empty() ? xdrg_schema_create(f.data(), nf, &s)
                                 : xdrg_schema_create_cond(f.data(), nf, c.data(), c.size(), &s);
        CHECK((st == XDRG_OK) == (s != nullptr));
        if (s) (void)xdrg_schema_fixed_size(s);
        xdrg_schema_destroy(s);
    }
    CHECK(xdrg_schema_create(nullptr, 3, nullptr) == XDRG_E_INVAL);
    for (int st = -2; st < 14; ++st) CHECK(xdrg_status_string(st) != nullptr);
    // every entry point refuses a NULL context / schema without touching a device
    uint64_t len = 0, fb = 0;
    int err = 0;
    CHECK(xdrg_encode_batch(nullptr, nullptr, nullptr, 1, nullptr, 0, nullptr, 0, &len) == XDRG_E_INVAL);
    CHECK(xdrg_decode_batch(nullptr, nullptr, nullptr, 0, nullptr, 1, nullptr, 0, &fb, &err) == XDRG_E_INVAL);
    CHECK(xdrg_frame_scan(nullptr, nullptr, 0, nullptr, 0, &len) == XDRG_E_INVAL);
    CHECK(xdrg_ctx_destroy(nullptr) == XDRG_OK);
    CHECK(std::strlen(xdrg_last_error(nullptr)) == 0);
}

static void buffers(std::mt19937_64 &rng) {
    for (int composite = 0; composite < 2; ++composite) {
        XdrBuffer b(XdrBuffer::kInitialSize, composite);
        std::vector<uint8_t> shadow;
        size_t cap = b.capacity();
        for (int r = 0; r < 200; ++r) {
            std::vector<uint8_t> chunk(rng() % 3000);
            for (auto &x : chunk) x = (uint8_t)rng();
            const size_t before = b.remaining();
            b.put(chunk.data(), chunk.size());
            if (chunk.size() > before) {   // grew exactly as Xdr.ensureCapacity does
                CHECK(b.capacity() == std::max(cap * 3 / 2 + 1, cap + chunk.size()));
                if (composite) CHECK(b.chunks() >= 2);
                cap = b.capacity();
            }
            shadow.insert(shadow.end(), chunk.begin(), chunk.end());
        }
        b.flip();
        CHECK(b.bytes() == shadow);
        CHECK(b.isComposite() == (composite != 0) && (composite || b.chunks() == 1));
    }
}

int main() {
    std::mt19937_64 rng(0x0DCAC4E5);
    schemas(rng);
    buffers(rng);
    std::printf("san_host: ok\n");
    return 0;
}
