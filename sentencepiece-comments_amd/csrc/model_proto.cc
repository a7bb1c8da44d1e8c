// Wire-format reader for ModelProto (see model_proto.h).
#include "model_proto.h"

#include <cstring>

namespace spm_amd {
namespace {

// One length-delimited region of the buffer.
class Wire {
 public:
  Wire(const uint8_t *b, size_t n) : cur_(b), end_(b + n) {}
  bool more() const { return good_ && cur_ < end_; }
  bool good() const { return good_; }

  bool Tag(uint32_t *field, uint32_t *wire_type) {
    uint64_t t;
    if (!Varint(&t)) return false;
    *field = static_cast<uint32_t>(t >> 3);
    *wire_type = static_cast<uint32_t>(t & 7u);
    return *field != 0 || Fail();
  }
  bool Varint(uint64_t *v) {
    uint64_t r = 0;
    for (int shift = 0; shift < 64 && cur_ < end_; shift += 7) {
      const uint8_t b = *cur_++;
      r |= static_cast<uint64_t>(b & 0x7Fu) << shift;
      if ((b & 0x80u) == 0) {
        *v = r;
        return true;
      }
    }
    return Fail();
  }
  bool Bytes(const uint8_t **p, size_t *n) {
    uint64_t len;
    if (!Varint(&len) || len > static_cast<uint64_t>(end_ - cur_)) return Fail();
    *p = cur_;
    *n = static_cast<size_t>(len);
    cur_ += len;
    return true;
  }
  bool String(std::string *s) {
    const uint8_t *p;
    size_t n;
    if (!Bytes(&p, &n)) return false;
    s->assign(reinterpret_cast<const char *>(p), n);
    return true;
  }
  bool Fixed32(uint32_t *v) {
    if (end_ - cur_ < 4) return Fail();
    std::memcpy(v, cur_, 4);
    cur_ += 4;
    return true;
  }
  bool Bool(bool *b) {
    uint64_t v;
    if (!Varint(&v)) return false;
    *b = v != 0;
    return true;
  }
  bool Skip(uint32_t wire_type) {
    uint64_t v;
    uint32_t f;
    const uint8_t *p;
    size_t n;
    switch (wire_type) {
      case 0: return Varint(&v);
      case 1:
        if (end_ - cur_ < 8) return Fail();
        cur_ += 8;
        return true;
      case 2: return Bytes(&p, &n);
      case 5: return Fixed32(&f);
      default: return Fail();
    }
  }

 private:
  bool Fail() {
    good_ = false;
    return false;
  }
  const uint8_t *cur_;
  const uint8_t *end_;
  bool good_ = true;
};

bool ParsePieceRec(const uint8_t *b, size_t n, PieceRec *out) {
  Wire w(b, n);
  uint32_t f, wt;
  while (w.more() && w.Tag(&f, &wt)) {
    if (f == 1 && wt == 2) {
      w.String(&out->piece);
    } else if (f == 2 && wt == 5) {
      uint32_t bits;
      if (w.Fixed32(&bits)) std::memcpy(&out->score, &bits, 4);
    } else if (f == 3 && wt == 0) {
      uint64_t t;
      if (w.Varint(&t) && t >= kNormal && t <= kUnused) out->type = static_cast<int32_t>(t);
    } else {
      w.Skip(wt);
    }
  }
  return w.good();
}

bool ParseTrainerSpec(const uint8_t *b, size_t n, TrainerSpecView *ts) {
  Wire w(b, n);
  uint32_t f, wt;
  while (w.more() && w.Tag(&f, &wt)) {
    if (f == 3 && wt == 0) {
      uint64_t t;
      if (w.Varint(&t) && t >= kUnigram && t <= kChar) ts->model_type = static_cast<int32_t>(t);
    } else if (f == 24 && wt == 0) {
      w.Bool(&ts->treat_whitespace_as_suffix);
    } else if (f == 44 && wt == 2) {
      ts->has_unk_surface = w.String(&ts->unk_surface);
    } else if (f == 45 && wt == 2) {
      w.String(&ts->unk_piece);
    } else if (f == 46 && wt == 2) {
      w.String(&ts->bos_piece);
    } else if (f == 47 && wt == 2) {
      w.String(&ts->eos_piece);
    } else if (f == 48 && wt == 2) {
      w.String(&ts->pad_piece);
    } else {
      w.Skip(wt);
    }
  }
  return w.good();
}

bool ParseNormalizerSpec(const uint8_t *b, size_t n, NormalizerSpecView *ns) {
  Wire w(b, n);
  uint32_t f, wt;
  while (w.more() && w.Tag(&f, &wt)) {
    if (f == 1 && wt == 2) w.String(&ns->name);
    else if (f == 2 && wt == 2) w.String(&ns->precompiled_charsmap);
    else if (f == 3 && wt == 0) w.Bool(&ns->add_dummy_prefix);
    else if (f == 4 && wt == 0) w.Bool(&ns->remove_extra_whitespaces);
    else if (f == 5 && wt == 0) w.Bool(&ns->escape_whitespaces);
    else w.Skip(wt);
  }
  return w.good();
}

bool ParseSelfTest(const uint8_t *b, size_t n,
                   std::vector<std::pair<std::string, std::string>> *out) {
  Wire w(b, n);
  uint32_t f, wt;
  while (w.more() && w.Tag(&f, &wt)) {
    if (f == 1 && wt == 2) {
      const uint8_t *p;
      size_t len;
      if (!w.Bytes(&p, &len)) break;
      Wire s(p, len);
      std::pair<std::string, std::string> sample;
      uint32_t g, gt;
      while (s.more() && s.Tag(&g, &gt)) {
        if (g == 1 && gt == 2) s.String(&sample.first);
        else if (g == 2 && gt == 2) s.String(&sample.second);
        else s.Skip(gt);
      }
      if (!s.good()) return false;
      out->push_back(std::move(sample));
    } else {
      w.Skip(wt);
    }
  }
  return w.good();
}

}  // namespace

bool ParseModelProto(const uint8_t *data, size_t len, ModelProtoView *out, std::string *err) {
  Wire w(data, len);
  uint32_t f, wt;
  bool ok = true;
  while (ok && w.more() && w.Tag(&f, &wt)) {
    const uint8_t *p = nullptr;
    size_t n = 0;
    if (wt == 2 && f >= 1 && f <= 4) {
      if (!w.Bytes(&p, &n)) break;
      switch (f) {
        case 1: {
          PieceRec rec;
          ok = ParsePieceRec(p, n, &rec);
          out->pieces.push_back(std::move(rec));
          break;
        }
        case 2: ok = ParseTrainerSpec(p, n, &out->trainer_spec); break;
        case 3: ok = ParseNormalizerSpec(p, n, &out->normalizer_spec); break;
        case 4: ok = ParseSelfTest(p, n, &out->self_test); break;
      }
    } else {
      w.Skip(wt);
    }
  }
  if (!ok || !w.good()) {
    if (err) *err = "cannot parse ModelProto";
    return false;
  }
  return true;
}

}  // namespace spm_amd
