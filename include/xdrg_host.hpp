// xdrg_host.hpp — C++ host-side mirror of the oncrpc4j XDR interface, built
// on the C-ABI of include/xdrg.h (libxdrg_host.so).
//
// The reference's per-field interface (paths under /root/reference/
// oncrpc4j-core/src/main/java/org/dcache/oncrpc4j/):
//   xdr/XdrEncodingStream.java:30-62   -> XdrEncodingStream
//   xdr/XdrDecodingStream.java:30-64   -> XdrDecodingStream
//   xdr/XdrAble.java:30-49             -> XdrAble
//   xdr/BadXdrOncRpcException.java:24  -> BadXdrOncRpcException
//   xdr/XdrInt.java, XdrLong.java, XdrString.java, XdrOpaque.java,
//   XdrBoolean.java, XdrVoid.java      -> the wrapper records below
//
// Same method names, argument meaning and error behaviour; the engine behind
// them is batched.  BatchXdrEncoder records the per-field calls of many
// records of one shape (the field tape of the first record is the schema)
// and encodes them in one GPU batch on flush(); BatchXdrDecoder decodes a
// whole stream in one GPU batch and then replays the per-field calls record
// by record.  Nothing here computes XDR on the CPU.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "xdrg.h"

namespace oncrpc4j {
namespace xdr {

// BadXdrOncRpcException (an IOException in the reference): "xdr stream too
// short" (Xdr.java:1030) / "corrupted xdr" (Xdr.java:1036).
class BadXdrOncRpcException : public std::runtime_error {
public:
    explicit BadXdrOncRpcException(const std::string &m) : std::runtime_error(m) {}
};

// Engine failure that has no reference counterpart (HIP error, capacity).
class XdrgError : public std::runtime_error {
public:
    XdrgError(int status, const std::string &m) : std::runtime_error(m), status(status) {}
    int status;
};

class XdrEncodingStream {   // XdrEncodingStream.java:30-57
public:
    virtual ~XdrEncodingStream() = default;
    virtual void beginEncoding() = 0;
    virtual void endEncoding() = 0;
    virtual void xdrEncodeInt(int32_t value) = 0;
    virtual void xdrEncodeIntVector(const std::vector<int32_t> &ints) = 0;
    virtual void xdrEncodeIntFixedVector(const std::vector<int32_t> &ints, int32_t length) = 0;
    virtual void xdrEncodeDynamicOpaque(const std::vector<uint8_t> &opaque) = 0;
    virtual void xdrEncodeOpaque(const std::vector<uint8_t> &opaque, int32_t len) = 0;
    virtual void xdrEncodeOpaque(const std::vector<uint8_t> &opaque, int32_t offset, int32_t len) = 0;
    virtual void xdrEncodeBoolean(bool b) = 0;
    virtual void xdrEncodeString(const std::string *str) = 0;   // nullptr encodes "" (Xdr.java:760)
    virtual void xdrEncodeLong(int64_t value) = 0;
    virtual void xdrEncodeLongVector(const std::vector<int64_t> &longs) = 0;
    virtual void xdrEncodeLongFixedVector(const std::vector<int64_t> &longs, int32_t length) = 0;
    virtual void xdrEncodeByteBuffer(const std::vector<uint8_t> &buf) = 0;
    virtual void xdrEncodeFloat(float value) = 0;
    virtual void xdrEncodeDouble(double value) = 0;
    virtual void xdrEncodeFloatVector(const std::vector<float> &value) = 0;
    virtual void xdrEncodeFloatFixedVector(const std::vector<float> &value, int32_t length) = 0;
    virtual void xdrEncodeDoubleVector(const std::vector<double> &value) = 0;
    virtual void xdrEncodeDoubleFixedVector(const std::vector<double> &value, int32_t length) = 0;
    virtual void xdrEncodeByteVector(const std::vector<int8_t> &value) = 0;
    virtual void xdrEncodeByteFixedVector(const std::vector<int8_t> &value, int32_t length) = 0;
    virtual void xdrEncodeByte(int8_t value) = 0;
    virtual void xdrEncodeShort(int16_t value) = 0;
    virtual void xdrEncodeShortVector(const std::vector<int16_t> &value) = 0;
    virtual void xdrEncodeShortFixedVector(const std::vector<int16_t> &value, int32_t length) = 0;
    void xdrEncodeString(const std::string &s) { xdrEncodeString(&s); }
};

class XdrDecodingStream {   // XdrDecodingStream.java:30-58
public:
    virtual ~XdrDecodingStream() = default;
    virtual void beginDecoding() = 0;
    virtual void endDecoding() = 0;
    virtual int32_t xdrDecodeInt() = 0;
    virtual std::vector<int32_t> xdrDecodeIntVector() = 0;
    virtual std::vector<int32_t> xdrDecodeIntFixedVector(int32_t length) = 0;
    virtual std::vector<uint8_t> xdrDecodeDynamicOpaque() = 0;
    virtual std::vector<uint8_t> xdrDecodeOpaque(int32_t length) = 0;
    virtual void xdrDecodeOpaque(uint8_t *data, int32_t offset, int32_t length) = 0;
    virtual bool xdrDecodeBoolean() = 0;
    virtual std::string xdrDecodeString() = 0;
    virtual int64_t xdrDecodeLong() = 0;
    virtual std::vector<int64_t> xdrDecodeLongVector() = 0;
    virtual std::vector<int64_t> xdrDecodeLongFixedVector(int32_t length) = 0;
    virtual std::vector<uint8_t> xdrDecodeByteBuffer() = 0;
    virtual float xdrDecodeFloat() = 0;
    virtual double xdrDecodeDouble() = 0;
    virtual std::vector<double> xdrDecodeDoubleVector() = 0;
    virtual std::vector<double> xdrDecodeDoubleFixedVector(int32_t length) = 0;
    virtual std::vector<float> xdrDecodeFloatVector() = 0;
    virtual std::vector<float> xdrDecodeFloatFixedVector(int32_t length) = 0;
    virtual std::vector<int8_t> xdrDecodeByteVector() = 0;
    virtual std::vector<int8_t> xdrDecodeByteFixedVector(int32_t length) = 0;
    virtual int8_t xdrDecodeByte() = 0;
    virtual int16_t xdrDecodeShort() = 0;
    virtual std::vector<int16_t> xdrDecodeShortVector() = 0;
    virtual std::vector<int16_t> xdrDecodeShortFixedVector(int32_t length) = 0;
};

class XdrAble {   // XdrAble.java:30-49
public:
    virtual ~XdrAble() = default;
    virtual void xdrEncode(XdrEncodingStream &xdr) const = 0;
    virtual void xdrDecode(XdrDecodingStream &xdr) = 0;
};

// ---- engine context ------------------------------------------------------
class Engine {
public:
    explicit Engine(int device = 0);
    ~Engine();
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    xdrg_ctx *ctx() const { return ctx_; }
    int device() const { return device_; }

private:
    xdrg_ctx *ctx_ = nullptr;
    int device_ = 0;
};

// ---- host staging buffer (Grizzly Buffer + GrizzlyMemoryManager) ------------
// The socket-side host buffer an encoded batch lands in, with the reference's
// growth semantics for callers that do not presize:
//   Xdr.ensureCapacity (Xdr.java:1020-1026): when fewer than `size` bytes
//     remain, newCapacity = max(capacity * 3 / 2 + 1, capacity + size);
//   GrizzlyMemoryManager.reallocate (GrizzlyMemoryManager.java:46-53): a
//     composite buffer appends a chunk of (newCapacity - capacity) bytes, any
//     other buffer is reallocated with a copy.
// position/limit/flip/clear/hasRemaining as the Grizzly Buffer the Xdr wraps.
class XdrBuffer {
public:
    static constexpr size_t kInitialSize = 1024;   // Xdr.INITIAL_XDR_SIZE (Xdr.java:49)
    explicit XdrBuffer(size_t capacity = kInitialSize, bool composite = false);

    size_t capacity() const { return cap_; }
    size_t position() const { return pos_; }
    size_t limit() const { return lim_; }
    size_t remaining() const { return lim_ - pos_; }
    bool hasRemaining() const { return pos_ < lim_; }
    bool isComposite() const { return composite_; }
    size_t chunks() const { return chunks_.size(); }   // composite parts (1 when contiguous)
    void clear() { pos_ = 0; lim_ = cap_; }            // beginEncoding (Xdr.java:137-140)
    void flip() { lim_ = pos_; pos_ = 0; }             // endEncoding (Xdr.java:143-146)
    void rewind() { pos_ = 0; }                        // begin/endDecoding (Xdr.java:122-134)

    // Xdr.ensureCapacity: grow (per the policy above) so that `size` more bytes fit.
    void ensureCapacity(size_t size);
    // GrizzlyMemoryManager.reallocate to exactly newCapacity (>= capacity()).
    void reallocate(size_t newCapacity);
    // Append bytes at the position (growing as ensureCapacity does).
    void put(const uint8_t *src, size_t len);
    // Bytes [from, from + len) into dst (across composite chunks).
    void get(size_t from, uint8_t *dst, size_t len) const;
    // Copy of [position, limit) (Xdr.getBytes, Xdr.java:998-1006).
    std::vector<uint8_t> bytes() const;

private:
    bool composite_;
    size_t cap_ = 0, pos_ = 0, lim_ = 0;
    std::vector<std::vector<uint8_t>> chunks_;
};

// A read-only view of bytes owned elsewhere (Xdr.asBuffer, Xdr.java:558-575:
// the buffer that backs the message, no copy).
struct BufferView {
    const uint8_t *data = nullptr;
    size_t size = 0;
};

// ---- batching encoder -------------------------------------------------------
// One record = the calls between beginEncoding() and endEncoding(), as
// RpcCall.acceptedReply drives one Xdr per message (RpcCall.java:323-343).
class BatchXdrEncoder final : public XdrEncodingStream {
public:
    explicit BatchXdrEncoder(Engine &engine);
    ~BatchXdrEncoder() override;

    void beginEncoding() override;
    void endEncoding() override;
    void xdrEncodeInt(int32_t value) override;
    void xdrEncodeIntVector(const std::vector<int32_t> &ints) override;
    void xdrEncodeIntFixedVector(const std::vector<int32_t> &ints, int32_t length) override;
    void xdrEncodeDynamicOpaque(const std::vector<uint8_t> &opaque) override;
    void xdrEncodeOpaque(const std::vector<uint8_t> &opaque, int32_t len) override;
    void xdrEncodeOpaque(const std::vector<uint8_t> &opaque, int32_t offset, int32_t len) override;
    void xdrEncodeBoolean(bool b) override;
    void xdrEncodeString(const std::string *str) override;
    using XdrEncodingStream::xdrEncodeString;
    void xdrEncodeLong(int64_t value) override;
    void xdrEncodeLongVector(const std::vector<int64_t> &longs) override;
    void xdrEncodeLongFixedVector(const std::vector<int64_t> &longs, int32_t length) override;
    void xdrEncodeByteBuffer(const std::vector<uint8_t> &buf) override;
    void xdrEncodeFloat(float value) override;
    void xdrEncodeDouble(double value) override;
    void xdrEncodeFloatVector(const std::vector<float> &value) override;
    void xdrEncodeFloatFixedVector(const std::vector<float> &value, int32_t length) override;
    void xdrEncodeDoubleVector(const std::vector<double> &value) override;
    void xdrEncodeDoubleFixedVector(const std::vector<double> &value, int32_t length) override;
    void xdrEncodeByteVector(const std::vector<int8_t> &value) override;
    void xdrEncodeByteFixedVector(const std::vector<int8_t> &value, int32_t length) override;
    void xdrEncodeByte(int8_t value) override;
    void xdrEncodeShort(int16_t value) override;
    void xdrEncodeShortVector(const std::vector<int16_t> &value) override;
    void xdrEncodeShortFixedVector(const std::vector<int16_t> &value, int32_t length) override;

    // Records recorded so far / the field tape (schema) of the batch.
    uint64_t records() const;
    const std::vector<xdrg_field> &schema() const;
    // Encode every recorded record on the GPU into one XDR stream (record i
    // at offsets[i]); `framed` prepends one RFC 1831 record mark per record
    // (GrizzlyRpcTransport.java:103-110).  Clears the batch.  The stream
    // lands in this encoder's host XdrBuffer, which starts at
    // XdrBuffer::kInitialSize and grows by the reference's policy when the
    // engine reports the batch does not fit (XDRG_E_CAPACITY + needed size).
    std::vector<uint8_t> flush(bool framed = false, std::vector<uint64_t> *offsets = nullptr);

    // Per-message access to the last flushed batch, the two ways the
    // reference hands an encoded message on (RpcGssCall.java:111-131,
    // GrizzlyRpcTransport.java:100): getBytes copies message i
    // (Xdr.getBytes, Xdr.java:998-1006) and throws std::logic_error
    // ("getBytes called while buffer in use", the reference's
    // IllegalStateException) between beginEncoding() and endEncoding();
    // asBuffer returns message i as a view of the stream (Xdr.asBuffer).
    std::vector<uint8_t> getBytes(uint64_t i) const;
    BufferView asBuffer(uint64_t i) const;
    uint64_t messages() const;            // messages in the last flushed batch
    const XdrBuffer &buffer() const;      // the stream's host buffer (growth history)

private:
    struct Impl;
    std::unique_ptr<Impl> p_;
};

// ---- batching decoder -------------------------------------------------------
class BatchXdrDecoder final : public XdrDecodingStream {
public:
    // The field tape of the records in the stream (e.g. BatchXdrEncoder::schema()
    // of a prototype, or schemaOf(prototype)).
    BatchXdrDecoder(Engine &engine, const std::vector<xdrg_field> &schema);
    ~BatchXdrDecoder() override;

    // Decode n records on the GPU.  rec_offsets (n+1) gives each record's
    // extent; empty = records back to back at the fixed size (fixed schemas).
    // Records before the first bad one decode; the bad record's
    // beginDecoding() throws what the reference would have thrown.
    void load(const std::vector<uint8_t> &xdr, uint64_t n, const std::vector<uint64_t> &rec_offsets = {},
              bool framed = false);
    uint64_t records() const;
    uint64_t firstBad() const;   // == records() when the whole stream decoded

    void beginDecoding() override;   // advances to the next record
    void endDecoding() override;
    // Xdr.hasMoreData (Xdr.java:152-154): bytes of the current record not yet
    // decoded (false before the first beginDecoding and past the last field).
    bool hasMoreData() const;
    int32_t xdrDecodeInt() override;
    std::vector<int32_t> xdrDecodeIntVector() override;
    std::vector<int32_t> xdrDecodeIntFixedVector(int32_t length) override;
    std::vector<uint8_t> xdrDecodeDynamicOpaque() override;
    std::vector<uint8_t> xdrDecodeOpaque(int32_t length) override;
    void xdrDecodeOpaque(uint8_t *data, int32_t offset, int32_t length) override;
    bool xdrDecodeBoolean() override;
    std::string xdrDecodeString() override;
    int64_t xdrDecodeLong() override;
    std::vector<int64_t> xdrDecodeLongVector() override;
    std::vector<int64_t> xdrDecodeLongFixedVector(int32_t length) override;
    std::vector<uint8_t> xdrDecodeByteBuffer() override;
    float xdrDecodeFloat() override;
    double xdrDecodeDouble() override;
    std::vector<double> xdrDecodeDoubleVector() override;
    std::vector<double> xdrDecodeDoubleFixedVector(int32_t length) override;
    std::vector<float> xdrDecodeFloatVector() override;
    std::vector<float> xdrDecodeFloatFixedVector(int32_t length) override;
    std::vector<int8_t> xdrDecodeByteVector() override;
    std::vector<int8_t> xdrDecodeByteFixedVector(int32_t length) override;
    int8_t xdrDecodeByte() override;
    int16_t xdrDecodeShort() override;
    std::vector<int16_t> xdrDecodeShortVector() override;
    std::vector<int16_t> xdrDecodeShortFixedVector(int32_t length) override;

private:
    struct Impl;
    std::unique_ptr<Impl> p_;
};

// The field tape of a record type, captured by recording one prototype's
// xdrEncode (no engine work).
std::vector<xdrg_field> schemaOf(const XdrAble &prototype);

// ---- the reference's wrapper records (xdr/Xdr*.java) ---------------------------
class XdrInt : public XdrAble {           // XdrInt.java:25-50
public:
    XdrInt() = default;
    explicit XdrInt(int32_t v) : value(v) {}
    int32_t intValue() const { return value; }
    void xdrEncode(XdrEncodingStream &x) const override { x.xdrEncodeInt(value); }
    void xdrDecode(XdrDecodingStream &x) override { value = x.xdrDecodeInt(); }
    int32_t value = 0;
};
class XdrLong : public XdrAble {          // XdrLong.java:6-27
public:
    XdrLong() = default;
    explicit XdrLong(int64_t v) : value(v) {}
    int64_t longValue() const { return value; }
    void xdrEncode(XdrEncodingStream &x) const override { x.xdrEncodeLong(value); }
    void xdrDecode(XdrDecodingStream &x) override { value = x.xdrDecodeLong(); }
    int64_t value = 0;
};
class XdrBoolean : public XdrAble {       // XdrBoolean.java:25-52
public:
    XdrBoolean() = default;
    explicit XdrBoolean(bool v) : value(v) {}
    bool booleanValue() const { return value; }
    void xdrEncode(XdrEncodingStream &x) const override { x.xdrEncodeBoolean(value); }
    void xdrDecode(XdrDecodingStream &x) override { value = x.xdrDecodeBoolean(); }
    bool value = false;
};
class XdrString : public XdrAble {        // XdrString.java:26-51
public:
    XdrString() = default;
    explicit XdrString(std::string v) : value(std::move(v)) {}
    const std::string &stringValue() const { return value; }
    void xdrEncode(XdrEncodingStream &x) const override { x.xdrEncodeString(&value); }
    void xdrDecode(XdrDecodingStream &x) override { value = x.xdrDecodeString(); }
    std::string value;
};
class XdrOpaque : public XdrAble {        // XdrOpaque.java:32-85 (dynamic opaque)
public:
    XdrOpaque() = default;
    explicit XdrOpaque(std::vector<uint8_t> v) : value(std::move(v)) {}
    const std::vector<uint8_t> &getOpaque() const { return value; }
    void xdrEncode(XdrEncodingStream &x) const override { x.xdrEncodeDynamicOpaque(value); }
    void xdrDecode(XdrDecodingStream &x) override { value = x.xdrDecodeDynamicOpaque(); }
    std::vector<uint8_t> value;
};

}  // namespace xdr
}  // namespace oncrpc4j
