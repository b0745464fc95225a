// xdr_buffer.cpp — XdrBuffer (include/xdrg_host.hpp): the host staging
// buffer of the C++ mirror, with the reference's growth semantics.
//   Xdr.ensureCapacity            Xdr.java:1020-1026
//   GrizzlyMemoryManager.reallocate GrizzlyMemoryManager.java:46-53
// Host-only code (no HIP): tests/test_sanitize.py also builds it under
// ASan/UBSan.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "xdrg_host.hpp"

namespace oncrpc4j {
namespace xdr {

XdrBuffer::XdrBuffer(size_t capacity, bool composite) : composite_(composite), cap_(capacity), lim_(capacity) {
    chunks_.emplace_back(capacity);
}

void XdrBuffer::ensureCapacity(size_t size) {
    if (remaining() >= size) return;
    const size_t grown = cap_ * 3 / 2 + 1;
    reallocate(std::max(grown, cap_ + size));
}

void XdrBuffer::reallocate(size_t newCapacity) {
    if (newCapacity < cap_) throw std::invalid_argument("reallocate below the current capacity");
    if (newCapacity == cap_) return;
    if (composite_) {
        chunks_.emplace_back(newCapacity - cap_);   // append an add-on chunk, no copy
    } else {
        std::vector<uint8_t> bigger(newCapacity);   // MemoryManager.reallocate: copy
        std::memcpy(bigger.data(), chunks_[0].data(), cap_);
        chunks_[0].swap(bigger);
    }
    // Grizzly keeps position; the limit of a buffer being written is its capacity
    if (lim_ == cap_) lim_ = newCapacity;
    cap_ = newCapacity;
}

void XdrBuffer::put(const uint8_t *src, size_t len) {
    ensureCapacity(len);
    size_t at = pos_, done = 0;
    for (auto &c : chunks_) {
        if (done == len) break;
        if (at >= c.size()) {
            at -= c.size();
            continue;
        }
        const size_t k = std::min(len - done, c.size() - at);
        std::memcpy(c.data() + at, src + done, k);
        done += k;
        at = 0;
    }
    pos_ += len;
}

void XdrBuffer::get(size_t from, uint8_t *dst, size_t len) const {
    if (from + len > cap_) throw std::out_of_range("XdrBuffer::get past the capacity");
    size_t at = from, done = 0;
    for (const auto &c : chunks_) {
        if (done == len) break;
        if (at >= c.size()) {
            at -= c.size();
            continue;
        }
        const size_t k = std::min(len - done, c.size() - at);
        std::memcpy(dst + done, c.data() + at, k);
        done += k;
        at = 0;
    }
}

std::vector<uint8_t> XdrBuffer::bytes() const {
    std::vector<uint8_t> v(remaining());
    if (!v.empty()) get(pos_, v.data(), v.size());
    return v;
}

}  // namespace xdr
}  // namespace oncrpc4j
