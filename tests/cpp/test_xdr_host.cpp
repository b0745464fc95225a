// test_xdr_host.cpp — the reference's XDR unit tests, restated against the
// C++ host mirror (include/xdrg_host.hpp) with the HIP engine behind it.
// Each case names the reference test it follows (paths under /root/reference/
// oncrpc4j-core/src/test/java/org/dcache/oncrpc4j/).  Needs a GPU.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include "xdrg_host.hpp"

using namespace oncrpc4j::xdr;

static int g_fail = 0;
#define EXPECT(c)                                                                       \
    do {                                                                                \
        if (!(c)) { std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); throw 1; } \
    } while (0)

static std::vector<uint8_t> hex(const char *h) {
    std::vector<uint8_t> v;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) v.push_back((uint8_t)std::stoi(std::string(h + i, 2), nullptr, 16));
    return v;
}

template <class E> static bool throws(const std::function<void()> &f) {
    try { f(); } catch (const E &) { return true; } catch (...) { return false; }
    return false;
}

static void run(const char *name, const std::function<void()> &f) {
    try {
        f();
        std::printf("ok %s\n", name);
    } catch (const std::exception &x) {
        std::printf("FAIL %s: %s\n", name, x.what());
        ++g_fail;
    } catch (...) {
        std::printf("FAIL %s\n", name);
        ++g_fail;
    }
}

// Encode one XdrAble as one record (new Xdr(..); beginEncoding; xdrEncode; endEncoding; getBytes)
static std::vector<uint8_t> encode1(Engine &e, const XdrAble &x) {
    BatchXdrEncoder enc(e);
    enc.beginEncoding();
    x.xdrEncode(enc);
    enc.endEncoding();
    return enc.flush();
}

// A two-field struct, as rpcgen emits for `struct mapping { int prog; ... }`
// (core/portmap/mapping.java:70-75) and rpcb (core/portmap/rpcb.java:95-102).
struct Rpcb : XdrAble {
    int32_t prog = 0, vers = 0;
    std::string netid, addr, owner;
    void xdrEncode(XdrEncodingStream &x) const override {
        x.xdrEncodeInt(prog); x.xdrEncodeInt(vers);
        x.xdrEncodeString(netid); x.xdrEncodeString(addr); x.xdrEncodeString(owner);
    }
    void xdrDecode(XdrDecodingStream &x) override {
        prog = x.xdrDecodeInt(); vers = x.xdrDecodeInt();
        netid = x.xdrDecodeString(); addr = x.xdrDecodeString(); owner = x.xdrDecodeString();
    }
};

// Every field kind the rpcgen vocabulary has.
struct Everything : XdrAble {
    int32_t i = 0; int64_t l = 0; float f = 0; double d = 0; bool b = false; int8_t by = 0; int16_t sh = 0;
    std::vector<int32_t> iv, ifv; std::vector<int64_t> lv, lfv; std::vector<float> fv, ffv;
    std::vector<double> dv, dfv; std::vector<int8_t> bv, bfv; std::vector<int16_t> sv, sfv;
    std::vector<uint8_t> op, fop; std::string s;
    void xdrEncode(XdrEncodingStream &x) const override {
        x.xdrEncodeInt(i); x.xdrEncodeLong(l); x.xdrEncodeFloat(f); x.xdrEncodeDouble(d); x.xdrEncodeBoolean(b);
        x.xdrEncodeByte(by); x.xdrEncodeShort(sh);
        x.xdrEncodeIntVector(iv); x.xdrEncodeIntFixedVector(ifv, 3); x.xdrEncodeLongVector(lv);
        x.xdrEncodeLongFixedVector(lfv, 2); x.xdrEncodeFloatVector(fv); x.xdrEncodeFloatFixedVector(ffv, 2);
        x.xdrEncodeDoubleVector(dv); x.xdrEncodeDoubleFixedVector(dfv, 1); x.xdrEncodeByteVector(bv);
        x.xdrEncodeByteFixedVector(bfv, 5); x.xdrEncodeShortVector(sv); x.xdrEncodeShortFixedVector(sfv, 3);
        x.xdrEncodeDynamicOpaque(op); x.xdrEncodeOpaque(fop, 7); x.xdrEncodeString(s);
    }
    void xdrDecode(XdrDecodingStream &x) override {
        i = x.xdrDecodeInt(); l = x.xdrDecodeLong(); f = x.xdrDecodeFloat(); d = x.xdrDecodeDouble();
        b = x.xdrDecodeBoolean(); by = x.xdrDecodeByte(); sh = x.xdrDecodeShort();
        iv = x.xdrDecodeIntVector(); ifv = x.xdrDecodeIntFixedVector(3); lv = x.xdrDecodeLongVector();
        lfv = x.xdrDecodeLongFixedVector(2); fv = x.xdrDecodeFloatVector(); ffv = x.xdrDecodeFloatFixedVector(2);
        dv = x.xdrDecodeDoubleVector(); dfv = x.xdrDecodeDoubleFixedVector(1); bv = x.xdrDecodeByteVector();
        bfv = x.xdrDecodeByteFixedVector(5); sv = x.xdrDecodeShortVector(); sfv = x.xdrDecodeShortFixedVector(3);
        op = x.xdrDecodeDynamicOpaque(); fop = x.xdrDecodeOpaque(7); s = x.xdrDecodeString();
    }
    bool operator==(const Everything &o) const {
        return i == o.i && l == o.l && std::memcmp(&f, &o.f, 4) == 0 && std::memcmp(&d, &o.d, 8) == 0 &&
               b == o.b && by == o.by && sh == o.sh && iv == o.iv && ifv == o.ifv && lv == o.lv && lfv == o.lfv &&
               fv == o.fv && ffv == o.ffv && dv == o.dv && dfv == o.dfv && bv == o.bv && bfv == o.bfv &&
               sv == o.sv && sfv == o.sfv && op == o.op && fop == o.fop && s == o.s;
    }
};

int main() {
    Engine e(0);

    run("XdrIntTest.testEncodeWellKnown (XdrIntTest.java:48-62)", [&] {
        EXPECT(encode1(e, XdrInt(17)) == hex("00000011"));
    });
    run("XdrIntTest.testDecodeWellKnown (XdrIntTest.java:66-80)", [&] {
        BatchXdrDecoder dec(e, schemaOf(XdrInt()));
        dec.load(hex("00000011"), 1);
        XdrInt x;
        dec.beginDecoding();
        x.xdrDecode(dec);
        EXPECT(x.intValue() == 17);
    });
    run("XdrLongTest.testEncodeWellKnown/testDecodeWellKnown (XdrLongTest.java:44-77)", [&] {
        EXPECT(encode1(e, XdrLong(297519060383110161LL)) == hex("04210002540b1411"));
        BatchXdrDecoder dec(e, schemaOf(XdrLong()));
        dec.load(hex("04210002540b1411"), 1);
        XdrLong x;
        dec.beginDecoding();
        x.xdrDecode(dec);
        EXPECT(x.longValue() == 297519060383110161LL);
    });
    run("XdrOpaqueTest.testEncodeWellKnown/testDecodeWellKnown (XdrOpaqueTest.java:86-144)", [&] {
        const auto data = hex("0c0a0f0e0b0a0b0e");
        EXPECT(encode1(e, XdrOpaque(data)) == hex("000000080c0a0f0e0b0a0b0e"));
        BatchXdrDecoder dec(e, schemaOf(XdrOpaque()));
        dec.load(hex("000000080c0a0f0e0b0a0b0e"), 1);
        XdrOpaque x;
        dec.beginDecoding();
        x.xdrDecode(dec);
        EXPECT(x.getOpaque() == data);
    });
    run("XdrTest.testGetBytes: boolean + long (XdrTest.java:360-376)", [&] {
        BatchXdrEncoder enc(e);
        enc.beginEncoding();
        enc.xdrEncodeBoolean(true);
        enc.xdrEncodeLong(17);
        enc.endEncoding();
        EXPECT(enc.flush() == hex("000000010000000000000011"));
    });
    run("XdrTest.testBadXdrWithInt: int encoded, long decoded (XdrTest.java:289-299)", [&] {
        BatchXdrDecoder dec(e, schemaOf(XdrLong()));
        dec.load(hex("00000001"), 1);
        EXPECT(dec.firstBad() == 0);
        EXPECT(throws<BadXdrOncRpcException>([&] { dec.beginDecoding(); }));
    });
    run("XdrTest.testBadXdrOnNegativeArraySize (XdrTest.java:328-341)", [&] {
        BatchXdrEncoder probe(e);
        probe.beginEncoding();
        probe.xdrEncodeIntVector({});
        probe.endEncoding();
        BatchXdrDecoder dec(e, probe.schema());
        dec.load(hex("fffffffe0000000100000002"), 1, {0, 12});
        try { dec.beginDecoding(); EXPECT(false); }
        catch (const BadXdrOncRpcException &x) { EXPECT(std::string(x.what()) == "corrupted xdr"); }
    });
    run("Xdr.xdrEncodeIntFixedVector length mismatch -> IllegalArgumentException (Xdr.java:624-631)", [&] {
        BatchXdrEncoder enc(e);
        enc.beginEncoding();
        EXPECT(throws<std::invalid_argument>([&] { enc.xdrEncodeIntFixedVector({1, 2, 3}, 4); }));
    });
    run("XdrTest string round trips incl. null -> \"\" (XdrTest.java:196-210)", [&] {
        BatchXdrEncoder enc(e);
        const std::string vals[] = {"", "a", "ab", "abc", "abcd", "abcde", "\xc3\xa9t\xc3\xa9"};
        for (const auto &v : vals) { enc.beginEncoding(); enc.xdrEncodeString(v); enc.endEncoding(); }
        enc.beginEncoding(); enc.xdrEncodeString(nullptr); enc.endEncoding();
        std::vector<uint64_t> offs;
        const auto bytes = enc.flush(false, &offs);
        EXPECT(bytes.size() == 4 * 8 + 0 + 4 + 4 + 4 + 4 + 8 + 8);
        BatchXdrDecoder dec(e, schemaOf(XdrString()));
        dec.load(bytes, 8, offs);
        for (const auto &v : vals) { dec.beginDecoding(); EXPECT(dec.xdrDecodeString() == v); }
        dec.beginDecoding();
        EXPECT(dec.xdrDecodeString().empty());
    });
    run("Float/Double NaN canonicalisation (Xdr.java:674-687)", [&] {
        BatchXdrEncoder enc(e);
        uint32_t nanbits = 0x7f800123u;
        float f;
        std::memcpy(&f, &nanbits, 4);
        enc.beginEncoding(); enc.xdrEncodeFloat(f); enc.xdrEncodeDouble(std::nan("7")); enc.endEncoding();
        EXPECT(enc.flush() == hex("7fc000007ff8000000000000"));
    });
    run("rpcb batch of 50000 records, raw and record-marked (portmap/rpcb.java:95-102)", [&] {
        std::mt19937 rng(7);
        std::vector<Rpcb> recs(50000);
        for (auto &r : recs) {
            r.prog = (int32_t)rng(); r.vers = (int32_t)(rng() % 5);
            r.netid = std::string(rng() % 6, 't'); r.addr = std::string(rng() % 40, '1');
            r.owner = std::string(rng() % 9, 'o');
        }
        for (bool framed : {false, true}) {
            BatchXdrEncoder enc(e);
            for (const auto &r : recs) { enc.beginEncoding(); r.xdrEncode(enc); enc.endEncoding(); }
            std::vector<uint64_t> offs;
            const auto bytes = enc.flush(framed, &offs);
            EXPECT(offs.size() == recs.size() + 1 && offs.back() == bytes.size());
            // spot-check record 1234 by hand: [mark] prog vers netid addr owner
            const uint8_t *p = bytes.data() + offs[1234];
            if (framed) {
                const uint32_t m = ((uint32_t)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3];
                EXPECT(m == (0x80000000u | (uint32_t)(offs[1235] - offs[1234] - 4)));
                p += 4;
            }
            const uint32_t prog = ((uint32_t)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3];
            EXPECT((int32_t)prog == recs[1234].prog);
            BatchXdrDecoder dec(e, schemaOf(Rpcb()));
            dec.load(bytes, recs.size(), offs, framed);
            EXPECT(dec.firstBad() == recs.size());
            for (const auto &want : recs) {
                Rpcb got;
                dec.beginDecoding();
                got.xdrDecode(dec);
                EXPECT(got.prog == want.prog && got.vers == want.vers && got.netid == want.netid &&
                       got.addr == want.addr && got.owner == want.owner);
            }
        }
    });
    run("every field kind, 3000 records round trip", [&] {
        std::mt19937 rng(11);
        auto rnd = [&](size_t k) { return (size_t)(rng() % k); };
        std::vector<Everything> recs(3000);
        for (auto &r : recs) {
            r.i = (int32_t)rng(); r.l = ((int64_t)rng() << 32) | rng(); r.f = (float)rng() / 7.f;
            r.d = (double)rng() / 3.0; r.b = rng() & 1; r.by = (int8_t)rng(); r.sh = (int16_t)rng();
            r.iv.resize(rnd(5)); for (auto &x : r.iv) x = (int32_t)rng();
            r.ifv = {(int32_t)rng(), 1, 2};
            r.lv.resize(rnd(4)); for (auto &x : r.lv) x = (int64_t)rng() * 977;
            r.lfv = {(int64_t)rng(), -1};
            r.fv.resize(rnd(4)); for (auto &x : r.fv) x = (float)rng();
            r.ffv = {1.5f, -2.f};
            r.dv.resize(rnd(3)); for (auto &x : r.dv) x = (double)rng();
            r.dfv = {3.25};
            r.bv.resize(rnd(6)); for (auto &x : r.bv) x = (int8_t)rng();
            r.bfv = {1, -1, 2, -2, 3};
            r.sv.resize(rnd(5)); for (auto &x : r.sv) x = (int16_t)rng();
            r.sfv = {-7, 7, 0};
            r.op.resize(rnd(13)); for (auto &x : r.op) x = (uint8_t)rng();
            r.fop.resize(7); for (auto &x : r.fop) x = (uint8_t)rng();
            r.s = std::string(rnd(11), 'z');
        }
        BatchXdrEncoder enc(e);
        for (const auto &r : recs) { enc.beginEncoding(); r.xdrEncode(enc); enc.endEncoding(); }
        std::vector<uint64_t> offs;
        const auto bytes = enc.flush(false, &offs);
        BatchXdrDecoder dec(e, schemaOf(Everything()));
        dec.load(bytes, recs.size(), offs);
        for (const auto &want : recs) {
            Everything got;
            dec.beginDecoding();
            got.xdrDecode(dec);
            EXPECT(got == want);
        }
    });
    run("record shape change inside a batch -> flush first", [&] {
        BatchXdrEncoder enc(e);
        enc.beginEncoding(); enc.xdrEncodeInt(1); enc.endEncoding();
        enc.beginEncoding();
        EXPECT(throws<std::logic_error>([&] { enc.xdrEncodeLong(2); }));
    });

    // XdrTest.testGetBytes (ctest/xdr/XdrTest.java:360-376): bool true + long 17
    // -> 12 bytes; getBytes while encoding -> IllegalStateException.
    run("getBytes / asBuffer per message, IllegalStateException while in use", [&] {
        BatchXdrEncoder enc(e);
        for (int i = 0; i < 3; ++i) {
            enc.beginEncoding();
            enc.xdrEncodeBoolean(true);
            enc.xdrEncodeLong(17 + i);
            enc.endEncoding();
        }
        const auto all = enc.flush();
        EXPECT(enc.messages() == 3 && all.size() == 36);
        EXPECT(enc.getBytes(0) == hex("00000001" "0000000000000011"));
        EXPECT(enc.getBytes(2) == hex("00000001" "0000000000000013"));
        const BufferView v = enc.asBuffer(1);
        EXPECT(v.size == 12 && std::memcmp(v.data, all.data() + 12, 12) == 0);
        enc.beginEncoding();
        EXPECT(throws<std::logic_error>([&] { (void)enc.getBytes(0); }));
        enc.xdrEncodeBoolean(false);
        enc.xdrEncodeLong(0);
        enc.endEncoding();
        EXPECT(enc.getBytes(0).size() == 12);   // not in use again: the last flushed batch
        EXPECT(throws<std::out_of_range>([&] { (void)enc.getBytes(3); }));
    });
    // Xdr.ensureCapacity growth (Xdr.java:1020-1026) through the engine's
    // capacity report: a 1 KiB initial buffer grows once to fit the batch.
    run("flush grows the host buffer by the reference policy", [&] {
        BatchXdrEncoder enc(e);
        const std::vector<uint8_t> blob(3000, 0x5a);
        for (int i = 0; i < 5; ++i) {
            enc.beginEncoding();
            enc.xdrEncodeInt(i);
            enc.xdrEncodeDynamicOpaque(blob);
            enc.endEncoding();
        }
        const size_t need = 5 * (4 + 4 + 3000);
        const auto out = enc.flush();
        EXPECT(out.size() == need);
        const size_t want_cap = std::max<size_t>(XdrBuffer::kInitialSize * 3 / 2 + 1, XdrBuffer::kInitialSize + need);
        EXPECT(enc.buffer().capacity() == want_cap);
        EXPECT(enc.buffer().remaining() == need && enc.buffer().bytes() == out);
    });
    // Xdr.hasMoreData (Xdr.java:152-154) while a record's fields are replayed
    run("hasMoreData over a record's fields", [&] {
        BatchXdrEncoder enc(e);
        enc.beginEncoding(); enc.xdrEncodeInt(7); enc.xdrEncodeString(std::string("ab")); enc.endEncoding();
        std::vector<uint64_t> offs;
        const auto bytes = enc.flush(false, &offs);
        BatchXdrDecoder dec(e, {{XDRG_T_INT, XDRG_K_SCALAR, 0, 0}, {XDRG_T_STRING, XDRG_K_DYNAMIC, 0, 0}});
        dec.load(bytes, 1, offs);
        EXPECT(!dec.hasMoreData());
        dec.beginDecoding();
        EXPECT(dec.hasMoreData());
        EXPECT(dec.xdrDecodeInt() == 7);
        EXPECT(dec.hasMoreData());
        EXPECT(dec.xdrDecodeString() == "ab");
        EXPECT(!dec.hasMoreData());
    });

    if (g_fail) {
        std::printf("%d FAILED\n", g_fail);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
