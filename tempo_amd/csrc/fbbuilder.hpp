// fbbuilder.hpp — back-to-front flatbuffer builder with the exact placement rules
// of the Go runtime the reference writes with
// (vendor/github.com/google/flatbuffers/go/builder.go: Prep :214-235, WriteVtable
// :105-190, StartVector/EndVector :294-316, CreateString/CreateSharedString
// :319-346, finish :598-614). Offsets are relative to the buffer end, so buffer
// growth policy does not change the bytes produced.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace tsg {

class FBBuilder {
 public:
  explicit FBBuilder(size_t initial = 1024) { buf_.resize(initial ? initial : 1); head_ = uint32_t(buf_.size()); }

  void reset() {
    head_ = uint32_t(buf_.size());
    minalign_ = 1;
    vtables_.clear();
    vtable_.clear();
    shared_.clear();
    nested_ = finished_ = false;
  }
  uint32_t offset() const { return uint32_t(buf_.size()) - head_; }

  void prep(size_t size, size_t additional) {
    if (size > minalign_) minalign_ = size;
    size_t align = (~(buf_.size() - head_ + additional) + 1) & (size - 1);
    while (head_ <= align + size + additional) grow();
    pad(align);
  }
  void pad(size_t n) {
    for (size_t i = 0; i < n; i++) buf_[--head_] = 0;
  }
  void place_u8(uint8_t v) { buf_[--head_] = v; }
  void place_u16(uint16_t v) { head_ -= 2; std::memcpy(&buf_[head_], &v, 2); }
  void place_u32(uint32_t v) { head_ -= 4; std::memcpy(&buf_[head_], &v, 4); }
  void place_u64(uint64_t v) { head_ -= 8; std::memcpy(&buf_[head_], &v, 8); }
  void prepend_u16(uint16_t v) { prep(2, 0); place_u16(v); }
  void prepend_u32(uint32_t v) { prep(4, 0); place_u32(v); }
  void prepend_u64(uint64_t v) { prep(8, 0); place_u64(v); }
  void prepend_uoffset(uint32_t off) {
    prep(4, 0);
    place_u32(offset() - off + 4);
  }
  void prepend_soffset_zero() {
    prep(4, 0);
    place_u32(offset() + 4);  // PrependSOffsetT(0): off2 = Offset() - 0 + 4 (patched later)
  }

  void start_object(int numfields) {
    nested_ = true;
    vtable_.assign(size_t(numfields), 0);
    object_end_ = offset();
  }
  void slot(int i) { vtable_[size_t(i)] = offset(); }
  void prepend_uoffset_slot(int o, uint32_t x, uint32_t d) {
    if (x != d) {
      prepend_uoffset(x);
      slot(o);
    }
  }
  void prepend_u64_slot(int o, uint64_t x, uint64_t d) {
    if (x != d) {
      prepend_u64(x);
      slot(o);
    }
  }
  uint32_t end_object() {
    uint32_t n = write_vtable();
    nested_ = false;
    return n;
  }

  uint32_t start_vector(size_t elem, size_t n, size_t align) {
    nested_ = true;
    prep(4, elem * n);
    prep(align, elem * n);
    return offset();
  }
  uint32_t end_vector(size_t n) {
    place_u32(uint32_t(n));
    nested_ = false;
    return offset();
  }
  uint32_t create_string(std::string_view s) {
    nested_ = true;
    prep(4, s.size() + 1);
    place_u8(0);
    head_ -= uint32_t(s.size());
    if (!s.empty()) std::memcpy(&buf_[head_], s.data(), s.size());
    return end_vector(s.size());
  }
  uint32_t create_shared_string(const std::string &s) {
    auto it = shared_.find(s);
    if (it != shared_.end()) return it->second;
    uint32_t o = create_string(s);
    shared_.emplace(s, o);
    return o;
  }
  void finish(uint32_t root) {
    prep(minalign_, 4);
    prepend_uoffset(root);
    finished_ = true;
  }
  std::vector<uint8_t> finished_bytes() const { return std::vector<uint8_t>(buf_.begin() + head_, buf_.end()); }
  const uint8_t *data() const { return buf_.data() + head_; }
  size_t size() const { return buf_.size() - head_; }

 private:
  void grow() {
    size_t old = buf_.size();
    size_t nl = old * 2;
    std::vector<uint8_t> nb(nl, 0);
    std::memcpy(nb.data() + (nl - old), buf_.data(), old);
    buf_.swap(nb);
    head_ += uint32_t(nl - old);
  }
  static uint16_t rd16(const uint8_t *p) {
    uint16_t v;
    std::memcpy(&v, p, 2);
    return v;
  }
  uint32_t write_vtable() {
    prepend_soffset_zero();
    uint32_t object_offset = offset();
    size_t i = vtable_.size();
    while (i > 0 && vtable_[i - 1] == 0) i--;
    vtable_.resize(i);
    uint32_t existing = 0;
    for (size_t k = vtables_.size(); k-- > 0;) {
      uint32_t vt2 = vtables_[k];
      size_t vt2start = buf_.size() - vt2;
      uint16_t vt2len = rd16(&buf_[vt2start]);
      const uint8_t *v2 = &buf_[vt2start + 4];
      size_t v2n = (vt2len - 4) / 2;
      if (v2n != vtable_.size()) continue;
      bool eq = true;
      for (size_t a = 0; a < v2n && eq; a++) {
        uint16_t x = rd16(v2 + 2 * a);
        if (x == 0 && vtable_[a] == 0) continue;
        int32_t y = int32_t(object_offset) - int32_t(vtable_[a]);
        if (int32_t(x) != y) eq = false;
      }
      if (eq) {
        existing = vt2;
        break;
      }
    }
    if (existing == 0) {
      for (size_t k = vtable_.size(); k-- > 0;) {
        uint16_t off = vtable_[k] ? uint16_t(object_offset - vtable_[k]) : 0;
        prepend_u16(off);
      }
      prepend_u16(uint16_t(object_offset - object_end_));
      prepend_u16(uint16_t((vtable_.size() + 2) * 2));
      size_t object_start = buf_.size() - object_offset;
      int32_t so = int32_t(offset()) - int32_t(object_offset);
      std::memcpy(&buf_[object_start], &so, 4);
      vtables_.push_back(offset());
    } else {
      size_t object_start = buf_.size() - object_offset;
      head_ = uint32_t(object_start);
      int32_t so = int32_t(existing) - int32_t(object_offset);
      std::memcpy(&buf_[head_], &so, 4);
    }
    vtable_.clear();
    return object_offset;
  }

  std::vector<uint8_t> buf_;
  uint32_t head_ = 0;
  size_t minalign_ = 1;
  std::vector<uint32_t> vtable_;
  uint32_t object_end_ = 0;
  std::vector<uint32_t> vtables_;
  std::unordered_map<std::string, uint32_t> shared_;
  bool nested_ = false, finished_ = false;
};

}  // namespace tsg
