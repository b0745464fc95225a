// xdr_batch.cpp — libxdrg_host.so: the C++ mirror of the oncrpc4j XDR
// interface (include/xdrg_host.hpp) over the C-ABI of include/xdrg.h.
//
// BatchXdrEncoder records per-field calls into native columns (host staging,
// the role Grizzly buffers play for the reference), BatchXdrDecoder replays
// decoded columns; all XDR arithmetic runs in libxdrgpu.so on the GPU.

#include <cstring>
#include <string>

#include "xdrg_host.hpp"

namespace oncrpc4j {
namespace xdr {

namespace {

[[noreturn]] void fail(int st, xdrg_ctx *ctx) {
    std::string msg = xdrg_status_string(st);
    if (st == XDRG_E_SHORT || st == XDRG_E_CORRUPT) throw BadXdrOncRpcException(msg);
    if (st == XDRG_E_FIXED_LEN) throw std::invalid_argument(msg);
    const char *d = ctx ? xdrg_last_error(ctx) : "";
    if (d && *d && msg != d) msg += std::string(" (") + d + ")";
    throw XdrgError(st, msg);
}
void check(int st, xdrg_ctx *ctx) {
    if (st) fail(st, ctx);
}

uint32_t native_size(uint32_t t) {
    switch (t) {
    case XDRG_T_INT: case XDRG_T_UINT: case XDRG_T_ENUM: case XDRG_T_FLOAT: return 4;
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_SHORT: return 2;
    default: return 1;
    }
}
uint32_t xdr_size(uint32_t t) {
    switch (t) {
    case XDRG_T_HYPER: case XDRG_T_UHYPER: case XDRG_T_DOUBLE: return 8;
    case XDRG_T_OPAQUE: case XDRG_T_STRING: return 1;
    default: return 4;
    }
}
uint64_t pad4(uint64_t n) { return (4 - (n & 3)) & 3; }

struct SchemaHandle {
    xdrg_schema *s = nullptr;
    explicit SchemaHandle(const std::vector<xdrg_field> &f) { check(xdrg_schema_create(f.data(), f.size(), &s), nullptr); }
    ~SchemaHandle() { xdrg_schema_destroy(s); }
};

struct Column {
    xdrg_field f;
    std::vector<uint8_t> data;       // native values
    std::vector<uint64_t> offsets;   // dynamic fields: n + 1 element offsets
};

bool same(const xdrg_field &a, const xdrg_field &b) {
    return a.type == b.type && a.kind == b.kind && (a.kind != XDRG_K_FIXED || a.count == b.count);
}

}  // namespace

// ---------------------------------------------------------------------------
Engine::Engine(int device) : device_(device) { check(xdrg_ctx_create(device, 0, &ctx_), nullptr); }
Engine::~Engine() { xdrg_ctx_destroy(ctx_); }

// ---------------------------------------------------------------------------
// Tape recorder: the field tape of one record, no values (schemaOf).
class TapeRecorder final : public XdrEncodingStream {
public:
    std::vector<xdrg_field> tape;
    void add(uint32_t t, uint32_t k, uint32_t c = 0) { tape.push_back({t, k, c, 0}); }
    void beginEncoding() override {}
    void endEncoding() override {}
    void xdrEncodeInt(int32_t) override { add(XDRG_T_INT, XDRG_K_SCALAR); }
    void xdrEncodeIntVector(const std::vector<int32_t> &) override { add(XDRG_T_INT, XDRG_K_DYNAMIC); }
    void xdrEncodeIntFixedVector(const std::vector<int32_t> &, int32_t n) override { add(XDRG_T_INT, XDRG_K_FIXED, n); }
    void xdrEncodeDynamicOpaque(const std::vector<uint8_t> &) override { add(XDRG_T_OPAQUE, XDRG_K_DYNAMIC); }
    void xdrEncodeOpaque(const std::vector<uint8_t> &, int32_t n) override { add(XDRG_T_OPAQUE, XDRG_K_FIXED, n); }
    void xdrEncodeOpaque(const std::vector<uint8_t> &, int32_t, int32_t n) override { add(XDRG_T_OPAQUE, XDRG_K_FIXED, n); }
    void xdrEncodeBoolean(bool) override { add(XDRG_T_BOOL, XDRG_K_SCALAR); }
    void xdrEncodeString(const std::string *) override { add(XDRG_T_STRING, XDRG_K_DYNAMIC); }
    void xdrEncodeLong(int64_t) override { add(XDRG_T_HYPER, XDRG_K_SCALAR); }
    void xdrEncodeLongVector(const std::vector<int64_t> &) override { add(XDRG_T_HYPER, XDRG_K_DYNAMIC); }
    void xdrEncodeLongFixedVector(const std::vector<int64_t> &, int32_t n) override { add(XDRG_T_HYPER, XDRG_K_FIXED, n); }
    void xdrEncodeByteBuffer(const std::vector<uint8_t> &) override { add(XDRG_T_OPAQUE, XDRG_K_DYNAMIC); }
    void xdrEncodeFloat(float) override { add(XDRG_T_FLOAT, XDRG_K_SCALAR); }
    void xdrEncodeDouble(double) override { add(XDRG_T_DOUBLE, XDRG_K_SCALAR); }
    void xdrEncodeFloatVector(const std::vector<float> &) override { add(XDRG_T_FLOAT, XDRG_K_DYNAMIC); }
    void xdrEncodeFloatFixedVector(const std::vector<float> &, int32_t n) override { add(XDRG_T_FLOAT, XDRG_K_FIXED, n); }
    void xdrEncodeDoubleVector(const std::vector<double> &) override { add(XDRG_T_DOUBLE, XDRG_K_DYNAMIC); }
    void xdrEncodeDoubleFixedVector(const std::vector<double> &, int32_t n) override { add(XDRG_T_DOUBLE, XDRG_K_FIXED, n); }
    void xdrEncodeByteVector(const std::vector<int8_t> &) override { add(XDRG_T_BYTE, XDRG_K_DYNAMIC); }
    void xdrEncodeByteFixedVector(const std::vector<int8_t> &, int32_t n) override { add(XDRG_T_BYTE, XDRG_K_FIXED, n); }
    void xdrEncodeByte(int8_t) override { add(XDRG_T_BYTE, XDRG_K_SCALAR); }
    void xdrEncodeShort(int16_t) override { add(XDRG_T_SHORT, XDRG_K_SCALAR); }
    void xdrEncodeShortVector(const std::vector<int16_t> &) override { add(XDRG_T_SHORT, XDRG_K_DYNAMIC); }
    void xdrEncodeShortFixedVector(const std::vector<int16_t> &, int32_t n) override { add(XDRG_T_SHORT, XDRG_K_FIXED, n); }
};

std::vector<xdrg_field> schemaOf(const XdrAble &prototype) {
    TapeRecorder t;
    prototype.xdrEncode(t);
    return t.tape;
}

// ---------------------------------------------------------------------------
struct BatchXdrEncoder::Impl {
    Engine *eng;
    std::vector<Column> cols;
    std::vector<xdrg_field> tape;
    bool have_tape = false, in_record = false;
    size_t field = 0;
    uint64_t n = 0;
    XdrBuffer buf;                      // host staging of the flushed stream (grows, never shrinks)
    std::vector<uint8_t> stream;        // the last flushed batch ...
    std::vector<uint64_t> offs;         // ... and its message offsets

    Column &next(uint32_t t, uint32_t k, uint32_t c = 0) {
        if (!in_record) throw std::logic_error("xdrEncode* outside beginEncoding()/endEncoding()");
        const xdrg_field f{t, k, k == XDRG_K_FIXED ? c : 0, 0};
        if (!have_tape) {
            tape.push_back(f);
            cols.push_back(Column{f, {}, {0}});
        } else if (field >= tape.size() || !same(tape[field], f)) {
            throw std::logic_error("record shape differs from the batch schema: flush() first");
        }
        return cols[field++];
    }
    template <class T> void scalar(uint32_t t, T v) {
        Column &c = next(t, XDRG_K_SCALAR);
        const size_t o = c.data.size();
        c.data.resize(o + sizeof(T));
        std::memcpy(c.data.data() + o, &v, sizeof(T));
    }
    template <class T> void fixed(uint32_t t, const T *v, int32_t len) {
        Column &c = next(t, XDRG_K_FIXED, (uint32_t)len);
        const size_t o = c.data.size();
        c.data.resize(o + sizeof(T) * (size_t)len);
        if (len) std::memcpy(c.data.data() + o, v, sizeof(T) * (size_t)len);
    }
    template <class T> void dynamic(uint32_t t, const T *v, size_t cnt) {
        Column &c = next(t, XDRG_K_DYNAMIC);
        const size_t o = c.data.size();
        c.data.resize(o + sizeof(T) * cnt);
        if (cnt) std::memcpy(c.data.data() + o, v, sizeof(T) * cnt);
        c.offsets.push_back(c.offsets.back() + cnt);
    }
};

BatchXdrEncoder::BatchXdrEncoder(Engine &engine) : p_(new Impl) { p_->eng = &engine; }
BatchXdrEncoder::~BatchXdrEncoder() = default;

void BatchXdrEncoder::beginEncoding() {   // Xdr.beginEncoding: a fresh record (Xdr.java:137-140)
    if (p_->in_record) throw std::logic_error("beginEncoding() inside a record");
    p_->in_record = true;
    p_->field = 0;
}
void BatchXdrEncoder::endEncoding() {
    if (!p_->in_record) throw std::logic_error("endEncoding() without beginEncoding()");
    if (p_->have_tape && p_->field != p_->tape.size())
        throw std::logic_error("record shape differs from the batch schema: flush() first");
    if (p_->tape.empty()) throw std::logic_error("a record needs at least one field");
    p_->in_record = false;
    p_->have_tape = true;
    ++p_->n;
}

#define FIXED_LEN_CHECK(v, len)                                                                  \
    if ((int64_t)(v).size() != (int64_t)(len))                                                   \
        throw std::invalid_argument("array size does not match protocol specification") /* Xdr.java:625-627 */

void BatchXdrEncoder::xdrEncodeInt(int32_t v) { p_->scalar(XDRG_T_INT, v); }
void BatchXdrEncoder::xdrEncodeIntVector(const std::vector<int32_t> &v) { p_->dynamic(XDRG_T_INT, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeIntFixedVector(const std::vector<int32_t> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_INT, v.data(), len);
}
void BatchXdrEncoder::xdrEncodeDynamicOpaque(const std::vector<uint8_t> &v) { p_->dynamic(XDRG_T_OPAQUE, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeOpaque(const std::vector<uint8_t> &v, int32_t len) { xdrEncodeOpaque(v, 0, len); }
void BatchXdrEncoder::xdrEncodeOpaque(const std::vector<uint8_t> &v, int32_t off, int32_t len) {
    if (off < 0 || len < 0 || (size_t)off + (size_t)len > v.size()) throw std::out_of_range("opaque range");
    p_->fixed(XDRG_T_OPAQUE, v.data() + off, len);
}
void BatchXdrEncoder::xdrEncodeBoolean(bool b) { p_->scalar<uint8_t>(XDRG_T_BOOL, b ? 1 : 0); }
void BatchXdrEncoder::xdrEncodeString(const std::string *s) {   // null -> "" (Xdr.java:760-763)
    static const std::string empty;
    const std::string &v = s ? *s : empty;
    p_->dynamic(XDRG_T_STRING, (const uint8_t *)v.data(), v.size());
}
void BatchXdrEncoder::xdrEncodeLong(int64_t v) { p_->scalar(XDRG_T_HYPER, v); }
void BatchXdrEncoder::xdrEncodeLongVector(const std::vector<int64_t> &v) { p_->dynamic(XDRG_T_HYPER, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeLongFixedVector(const std::vector<int64_t> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_HYPER, v.data(), len);
}
void BatchXdrEncoder::xdrEncodeByteBuffer(const std::vector<uint8_t> &v) { p_->dynamic(XDRG_T_OPAQUE, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeFloat(float v) { p_->scalar(XDRG_T_FLOAT, v); }
void BatchXdrEncoder::xdrEncodeDouble(double v) { p_->scalar(XDRG_T_DOUBLE, v); }
void BatchXdrEncoder::xdrEncodeFloatVector(const std::vector<float> &v) { p_->dynamic(XDRG_T_FLOAT, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeFloatFixedVector(const std::vector<float> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_FLOAT, v.data(), len);
}
void BatchXdrEncoder::xdrEncodeDoubleVector(const std::vector<double> &v) { p_->dynamic(XDRG_T_DOUBLE, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeDoubleFixedVector(const std::vector<double> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_DOUBLE, v.data(), len);
}
void BatchXdrEncoder::xdrEncodeByteVector(const std::vector<int8_t> &v) { p_->dynamic(XDRG_T_BYTE, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeByteFixedVector(const std::vector<int8_t> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_BYTE, v.data(), len);
}
void BatchXdrEncoder::xdrEncodeByte(int8_t v) { p_->scalar(XDRG_T_BYTE, v); }
void BatchXdrEncoder::xdrEncodeShort(int16_t v) { p_->scalar(XDRG_T_SHORT, v); }
void BatchXdrEncoder::xdrEncodeShortVector(const std::vector<int16_t> &v) { p_->dynamic(XDRG_T_SHORT, v.data(), v.size()); }
void BatchXdrEncoder::xdrEncodeShortFixedVector(const std::vector<int16_t> &v, int32_t len) {
    FIXED_LEN_CHECK(v, len);
    p_->fixed(XDRG_T_SHORT, v.data(), len);
}

uint64_t BatchXdrEncoder::records() const { return p_->n; }
const std::vector<xdrg_field> &BatchXdrEncoder::schema() const { return p_->tape; }

std::vector<uint8_t> BatchXdrEncoder::flush(bool framed, std::vector<uint64_t> *offsets) {
    if (p_->in_record) throw std::logic_error("flush() inside a record");
    Impl &m = *p_;
    std::vector<uint8_t> out;
    m.stream.clear();
    m.offs.assign(1, 0);
    if (!m.n) {
        if (offsets) offsets->assign(1, 0);
        return out;
    }
    SchemaHandle sch(m.tape);
    // Host columns straight into the engine (XDRG_HOST_PTRS: the context's
    // staging ring moves them chunk by chunk); the stream lands in the
    // XdrBuffer, grown as Xdr.ensureCapacity grows it (Xdr.java:1020-1026)
    // when the engine reports XDRG_E_CAPACITY and the bytes it needs.
    std::vector<xdrg_column> cols(m.cols.size());
    for (size_t k = 0; k < m.cols.size(); ++k) {
        Column &c = m.cols[k];
        if (c.data.empty()) c.data.resize(8);   // a valid pointer for empty columns
        cols[k].data = c.data.data();
        cols[k].stride = 0;
        cols[k].cap = c.data.size() / native_size(c.f.type);
        cols[k].offsets = c.f.kind == XDRG_K_DYNAMIC ? c.offsets.data() : nullptr;
    }
    m.offs.resize(m.n + 1);
    uint64_t len = 0;
    m.buf.clear();
    for (;;) {
        out.resize(m.buf.remaining());
        const int st = xdrg_encode_batch(m.eng->ctx(), sch.s, cols.data(), m.n, out.data(), out.size(),
                                         m.offs.data(), (framed ? XDRG_FRAME_RM : 0) | XDRG_HOST_PTRS, &len);
        if (st == XDRG_E_CAPACITY && len > m.buf.remaining()) {
            m.buf.ensureCapacity(len);
            continue;
        }
        check(st, m.eng->ctx());
        out.resize(len);
        break;
    }
    m.buf.put(out.data(), len);
    m.buf.flip();   // endEncoding (Xdr.java:143-146)
    if (offsets) *offsets = m.offs;
    m.stream = out;
    m.cols.clear();
    m.tape.clear();
    m.have_tape = false;
    m.n = 0;
    return out;
}

uint64_t BatchXdrEncoder::messages() const { return p_->offs.size() - 1; }
const XdrBuffer &BatchXdrEncoder::buffer() const { return p_->buf; }

std::vector<uint8_t> BatchXdrEncoder::getBytes(uint64_t i) const {
    // checkState(!_inUse, ...) (Xdr.java:999)
    if (p_->in_record) throw std::logic_error("getBytes called while buffer in use");
    if (i >= messages()) throw std::out_of_range("no such message in the last flushed batch");
    return std::vector<uint8_t>(p_->stream.begin() + (ptrdiff_t)p_->offs[i],
                                p_->stream.begin() + (ptrdiff_t)p_->offs[i + 1]);
}

BufferView BatchXdrEncoder::asBuffer(uint64_t i) const {
    if (i >= messages()) throw std::out_of_range("no such message in the last flushed batch");
    return BufferView{p_->stream.data() + p_->offs[i], (size_t)(p_->offs[i + 1] - p_->offs[i])};
}

// ---------------------------------------------------------------------------
struct BatchXdrDecoder::Impl {
    Engine *eng;
    std::vector<xdrg_field> tape;
    std::vector<Column> cols;
    uint64_t n = 0, first_bad = 0;
    int err = 0;
    int64_t rec = -1;
    size_t field = 0;

    const Column &next(uint32_t t, uint32_t k, uint32_t c = 0) {
        if (rec < 0 || (uint64_t)rec >= n) throw std::logic_error("xdrDecode* outside a record");
        const xdrg_field f{t, k, k == XDRG_K_FIXED ? c : 0, 0};
        if (field >= tape.size() || !same(tape[field], f))
            throw std::logic_error("decode call does not match the schema");
        return cols[field++];
    }
    template <class T> T scalar(uint32_t t) {
        const Column &c = next(t, XDRG_K_SCALAR);
        T v;
        std::memcpy(&v, c.data.data() + (size_t)rec * sizeof(T), sizeof(T));
        return v;
    }
    template <class T> std::vector<T> fixed(uint32_t t, int32_t len) {
        const Column &c = next(t, XDRG_K_FIXED, (uint32_t)len);
        std::vector<T> v((size_t)len);
        if (len) std::memcpy(v.data(), c.data.data() + (size_t)rec * len * sizeof(T), (size_t)len * sizeof(T));
        return v;
    }
    template <class T> std::vector<T> dynamic(uint32_t t) {
        const Column &c = next(t, XDRG_K_DYNAMIC);
        const uint64_t a = c.offsets[rec], b = c.offsets[rec + 1];
        std::vector<T> v(b - a);
        if (b > a) std::memcpy(v.data(), c.data.data() + a * sizeof(T), (b - a) * sizeof(T));
        return v;
    }
};

BatchXdrDecoder::BatchXdrDecoder(Engine &engine, const std::vector<xdrg_field> &schema) : p_(new Impl) {
    p_->eng = &engine;
    p_->tape = schema;
}
BatchXdrDecoder::~BatchXdrDecoder() = default;

void BatchXdrDecoder::load(const std::vector<uint8_t> &xdr, uint64_t n, const std::vector<uint64_t> &rec_offsets,
                           bool framed) {
    Impl &m = *p_;
    SchemaHandle sch(m.tape);
    // one record and no extents: the record is the whole buffer, as one Xdr
    // wraps one message (RpcMessageParserTCP.java:139)
    std::vector<uint64_t> one;
    const std::vector<uint64_t> *ro = &rec_offsets;
    if (rec_offsets.empty() && n == 1) {
        one = {0, (uint64_t)xdr.size()};
        ro = &one;
    }
    if (!ro->empty() && ro->size() != n + 1) throw std::invalid_argument("rec_offsets needs n + 1 entries");
    // host columns, filled by the engine through its staging ring (XDRG_HOST_PTRS)
    std::vector<xdrg_column> cols(m.tape.size());
    m.cols.assign(m.tape.size(), Column{});
    for (size_t k = 0; k < m.tape.size(); ++k) {
        const xdrg_field &f = m.tape[k];
        Column &c = m.cols[k];
        c.f = f;
        const uint32_t ns = native_size(f.type);
        if (f.kind == XDRG_K_DYNAMIC) {
            // a column cannot hold more elements than the stream has bytes
            const uint64_t cap = xdr.size() / (xdr_size(f.type) == 1 ? 1 : xdr_size(f.type)) + 1;
            c.data.resize(cap * ns);
            c.offsets.resize(n + 1);
            cols[k].cap = cap;
            cols[k].offsets = c.offsets.data();
        } else {
            const uint64_t cnt = f.kind == XDRG_K_FIXED ? f.count : 1;
            c.data.resize(n * cnt * ns + 8);
            cols[k].cap = 0;
            cols[k].offsets = nullptr;
        }
        cols[k].data = c.data.data();
        cols[k].stride = 0;
    }
    uint64_t fb = 0;
    int err = 0;
    static const uint8_t empty4[4] = {0, 0, 0, 0};
    const int st = xdrg_decode_batch(m.eng->ctx(), sch.s, xdr.empty() ? empty4 : xdr.data(), xdr.size(),
                                     ro->empty() ? nullptr : ro->data(), n, cols.data(),
                                     (framed ? XDRG_FRAME_RM : 0) | XDRG_HOST_PTRS, &fb, &err);
    if (st && st != XDRG_E_SHORT && st != XDRG_E_CORRUPT && st != XDRG_E_FRAME && st != XDRG_E_CAPACITY)
        fail(st, m.eng->ctx());
    m.n = n;
    m.first_bad = st ? fb : n;
    m.err = st ? err : 0;
    m.rec = -1;
}
uint64_t BatchXdrDecoder::records() const { return p_->n; }
uint64_t BatchXdrDecoder::firstBad() const { return p_->first_bad; }

void BatchXdrDecoder::beginDecoding() {
    Impl &m = *p_;
    ++m.rec;
    m.field = 0;
    if ((uint64_t)m.rec >= m.n) throw std::out_of_range("no more records");
    if ((uint64_t)m.rec >= m.first_bad) fail(m.err, m.eng->ctx());   // what the reference throws
}
void BatchXdrDecoder::endDecoding() {}

bool BatchXdrDecoder::hasMoreData() const {
    const Impl &m = *p_;
    if (m.rec < 0 || (uint64_t)m.rec >= m.n) return false;
    for (size_t k = m.field; k < m.tape.size(); ++k) {   // any remaining field with XDR bytes
        const xdrg_field &f = m.tape[k];
        if (f.kind != XDRG_K_FIXED || f.count) return true;   // scalars and length words are >= 4 bytes
    }
    return false;
}

int32_t BatchXdrDecoder::xdrDecodeInt() { return p_->scalar<int32_t>(XDRG_T_INT); }
std::vector<int32_t> BatchXdrDecoder::xdrDecodeIntVector() { return p_->dynamic<int32_t>(XDRG_T_INT); }
std::vector<int32_t> BatchXdrDecoder::xdrDecodeIntFixedVector(int32_t len) { return p_->fixed<int32_t>(XDRG_T_INT, len); }
std::vector<uint8_t> BatchXdrDecoder::xdrDecodeDynamicOpaque() { return p_->dynamic<uint8_t>(XDRG_T_OPAQUE); }
std::vector<uint8_t> BatchXdrDecoder::xdrDecodeOpaque(int32_t len) { return p_->fixed<uint8_t>(XDRG_T_OPAQUE, len); }
void BatchXdrDecoder::xdrDecodeOpaque(uint8_t *data, int32_t offset, int32_t len) {
    const std::vector<uint8_t> v = p_->fixed<uint8_t>(XDRG_T_OPAQUE, len);
    if (len) std::memcpy(data + offset, v.data(), (size_t)len);
}
bool BatchXdrDecoder::xdrDecodeBoolean() { return p_->scalar<uint8_t>(XDRG_T_BOOL) != 0; }
std::string BatchXdrDecoder::xdrDecodeString() {
    const std::vector<uint8_t> v = p_->dynamic<uint8_t>(XDRG_T_STRING);
    return std::string(v.begin(), v.end());
}
int64_t BatchXdrDecoder::xdrDecodeLong() { return p_->scalar<int64_t>(XDRG_T_HYPER); }
std::vector<int64_t> BatchXdrDecoder::xdrDecodeLongVector() { return p_->dynamic<int64_t>(XDRG_T_HYPER); }
std::vector<int64_t> BatchXdrDecoder::xdrDecodeLongFixedVector(int32_t len) { return p_->fixed<int64_t>(XDRG_T_HYPER, len); }
std::vector<uint8_t> BatchXdrDecoder::xdrDecodeByteBuffer() { return p_->dynamic<uint8_t>(XDRG_T_OPAQUE); }
float BatchXdrDecoder::xdrDecodeFloat() { return p_->scalar<float>(XDRG_T_FLOAT); }
double BatchXdrDecoder::xdrDecodeDouble() { return p_->scalar<double>(XDRG_T_DOUBLE); }
std::vector<double> BatchXdrDecoder::xdrDecodeDoubleVector() { return p_->dynamic<double>(XDRG_T_DOUBLE); }
std::vector<double> BatchXdrDecoder::xdrDecodeDoubleFixedVector(int32_t len) { return p_->fixed<double>(XDRG_T_DOUBLE, len); }
std::vector<float> BatchXdrDecoder::xdrDecodeFloatVector() { return p_->dynamic<float>(XDRG_T_FLOAT); }
std::vector<float> BatchXdrDecoder::xdrDecodeFloatFixedVector(int32_t len) { return p_->fixed<float>(XDRG_T_FLOAT, len); }
std::vector<int8_t> BatchXdrDecoder::xdrDecodeByteVector() { return p_->dynamic<int8_t>(XDRG_T_BYTE); }
std::vector<int8_t> BatchXdrDecoder::xdrDecodeByteFixedVector(int32_t len) { return p_->fixed<int8_t>(XDRG_T_BYTE, len); }
int8_t BatchXdrDecoder::xdrDecodeByte() { return p_->scalar<int8_t>(XDRG_T_BYTE); }
int16_t BatchXdrDecoder::xdrDecodeShort() { return p_->scalar<int16_t>(XDRG_T_SHORT); }
std::vector<int16_t> BatchXdrDecoder::xdrDecodeShortVector() { return p_->dynamic<int16_t>(XDRG_T_SHORT); }
std::vector<int16_t> BatchXdrDecoder::xdrDecodeShortFixedVector(int32_t len) { return p_->fixed<int16_t>(XDRG_T_SHORT, len); }

}  // namespace xdr
}  // namespace oncrpc4j
