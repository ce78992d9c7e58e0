// Janus packet wire codec (host C++; packets are ~50-200 B, no GPU benefit).
//
// Replaces msgpack.packb(d, use_bin_type=True) / msgpack.unpackb(b, raw=False) at
// backend/common/protocol.py:107 and :120 (msgpack >= 1.0.7, a third-party C
// extension). The encoder emits exactly the byte forms msgpack-python 1.x's packer
// chooses for the packet's value types (smallest fix/8/16/32 forms, str8 enabled by
// use_bin_type=True, Python float -> float64 0xcb); the decoder is a complete
// MessagePack reader into a flat pre-order node list that the Python mirror turns
// back into objects, raising on trailing bytes (msgpack's ExtraData), truncation
// and the reserved 0xc1 byte.
#include <cstring>
#include <vector>
#include "common.h"
#include "../../include/janus.h"

namespace janus {
namespace {

struct Out {
  uint8_t* p;
  size_t cap, n = 0;
  bool overflow = false;
  void put(uint8_t b) {
    if (n < cap) p[n] = b; else overflow = true;
    ++n;
  }
  void be(uint64_t v, int bytes) {
    for (int k = bytes - 1; k >= 0; --k) put((uint8_t)(v >> (8 * k)));
  }
  void raw(const char* s, size_t len) {
    for (size_t k = 0; k < len; ++k) put((uint8_t)s[k]);
  }
};

void pack_str(Out& o, const char* s, size_t len) {
  if (len < 32) o.put((uint8_t)(0xa0 | len));
  else if (len < 256) { o.put(0xd9); o.be(len, 1); }
  else if (len < 65536) { o.put(0xda); o.be(len, 2); }
  else if (len <= 0xffffffffull) { o.put(0xdb); o.be(len, 4); }
  else throw Error("str too long for msgpack");
  o.raw(s, len);
}

void pack_int(Out& o, int64_t v) {
  if (v >= 0) {
    const uint64_t u = (uint64_t)v;
    if (u < 128) o.put((uint8_t)u);
    else if (u <= 0xff) { o.put(0xcc); o.be(u, 1); }
    else if (u <= 0xffff) { o.put(0xcd); o.be(u, 2); }
    else if (u <= 0xffffffffull) { o.put(0xce); o.be(u, 4); }
    else { o.put(0xcf); o.be(u, 8); }
  } else {
    if (v >= -32) o.put((uint8_t)(int8_t)v);
    else if (v >= -128) { o.put(0xd0); o.be((uint8_t)(int8_t)v, 1); }
    else if (v >= -32768) { o.put(0xd1); o.be((uint16_t)(int16_t)v, 2); }
    else if (v >= -2147483648ll) { o.put(0xd2); o.be((uint32_t)(int32_t)v, 4); }
    else { o.put(0xd3); o.be((uint64_t)v, 8); }
  }
}

void pack_uint(Out& o, uint64_t u) {
  if (u <= (uint64_t)INT64_MAX) pack_int(o, (int64_t)u);
  else { o.put(0xcf); o.be(u, 8); }
}

void pack_map_header(Out& o, size_t n) {
  if (n < 16) o.put((uint8_t)(0x80 | n));
  else if (n < 65536) { o.put(0xde); o.be(n, 2); }
  else { o.put(0xdf); o.be(n, 4); }
}

void pack_value(Out& o, const janus_value& v) {
  switch (v.type) {
    case JANUS_VAL_NIL: o.put(0xc0); break;
    case JANUS_VAL_BOOL: o.put(v.i ? 0xc3 : 0xc2); break;
    case JANUS_VAL_INT: pack_int(o, v.i); break;
    case JANUS_VAL_UINT: pack_uint(o, (uint64_t)v.i); break;
    case JANUS_VAL_FLOAT: {
      uint64_t bits;
      std::memcpy(&bits, &v.f, 8);
      o.put(0xcb);
      o.be(bits, 8);
      break;
    }
    case JANUS_VAL_STR: pack_str(o, v.s, v.len); break;
    default: throw Error("unsupported janus_value type " + std::to_string(v.type));
  }
}

// ---------------------------------------------------------------- decoder
struct In {
  const uint8_t* p;
  size_t len, pos = 0;
  uint8_t u8() {
    if (pos >= len) throw Error("msgpack: truncated input");
    return p[pos++];
  }
  uint64_t be(int bytes) {
    if (pos + bytes > len) throw Error("msgpack: truncated input");
    uint64_t v = 0;
    for (int k = 0; k < bytes; ++k) v = (v << 8) | p[pos++];
    return v;
  }
  size_t take(size_t n) {
    if (n > len - pos) throw Error("msgpack: truncated input");
    size_t at = pos;
    pos += n;
    return at;
  }
};

struct Nodes {
  janus_mp_node* out;
  size_t cap, n = 0;
  janus_mp_node& add() {
    if (n >= cap) throw Error("msgpack: node capacity exceeded");
    janus_mp_node& nd = out[n++];
    std::memset(&nd, 0, sizeof(nd));
    return nd;
  }
};

void decode(In& in, Nodes& nodes, int depth) {
  if (depth > 512) throw Error("msgpack: nesting too deep");
  const uint8_t b = in.u8();
  janus_mp_node& nd = nodes.add();
  auto str = [&](size_t n, int type) { nd.type = type; nd.len = n; nd.offset = in.take(n); };
  auto children = [&](size_t n, int type, size_t per) {
    nd.type = type;
    nd.len = n;
    for (size_t k = 0; k < n * per; ++k) decode(in, nodes, depth + 1);
  };
  if (b <= 0x7f) { nd.type = JANUS_VAL_INT; nd.i = b; }
  else if (b >= 0xe0) { nd.type = JANUS_VAL_INT; nd.i = (int8_t)b; }
  else if ((b & 0xf0) == 0x80) children(b & 0x0f, JANUS_VAL_MAP, 2);
  else if ((b & 0xf0) == 0x90) children(b & 0x0f, JANUS_VAL_ARRAY, 1);
  else if ((b & 0xe0) == 0xa0) str(b & 0x1f, JANUS_VAL_STR);
  else switch (b) {
    case 0xc0: nd.type = JANUS_VAL_NIL; break;
    case 0xc2: nd.type = JANUS_VAL_BOOL; nd.i = 0; break;
    case 0xc3: nd.type = JANUS_VAL_BOOL; nd.i = 1; break;
    case 0xc4: str(in.be(1), JANUS_VAL_BIN); break;
    case 0xc5: str(in.be(2), JANUS_VAL_BIN); break;
    case 0xc6: str(in.be(4), JANUS_VAL_BIN); break;
    case 0xca: {
      uint32_t u = (uint32_t)in.be(4);
      float f;
      std::memcpy(&f, &u, 4);
      nd.type = JANUS_VAL_FLOAT;
      nd.f = f;
      break;
    }
    case 0xcb: {
      uint64_t u = in.be(8);
      std::memcpy(&nd.f, &u, 8);
      nd.type = JANUS_VAL_FLOAT;
      break;
    }
    case 0xcc: nd.type = JANUS_VAL_INT; nd.i = (int64_t)in.be(1); break;
    case 0xcd: nd.type = JANUS_VAL_INT; nd.i = (int64_t)in.be(2); break;
    case 0xce: nd.type = JANUS_VAL_INT; nd.i = (int64_t)in.be(4); break;
    case 0xcf: {
      uint64_t u = in.be(8);
      nd.type = u > (uint64_t)INT64_MAX ? JANUS_VAL_UINT : JANUS_VAL_INT;
      nd.i = (int64_t)u;
      break;
    }
    case 0xd0: nd.type = JANUS_VAL_INT; nd.i = (int8_t)in.be(1); break;
    case 0xd1: nd.type = JANUS_VAL_INT; nd.i = (int16_t)in.be(2); break;
    case 0xd2: nd.type = JANUS_VAL_INT; nd.i = (int32_t)in.be(4); break;
    case 0xd3: nd.type = JANUS_VAL_INT; nd.i = (int64_t)in.be(8); break;
    case 0xd9: str(in.be(1), JANUS_VAL_STR); break;
    case 0xda: str(in.be(2), JANUS_VAL_STR); break;
    case 0xdb: str(in.be(4), JANUS_VAL_STR); break;
    case 0xdc: children(in.be(2), JANUS_VAL_ARRAY, 1); break;
    case 0xdd: children(in.be(4), JANUS_VAL_ARRAY, 1); break;
    case 0xde: children(in.be(2), JANUS_VAL_MAP, 2); break;
    case 0xdf: children(in.be(4), JANUS_VAL_MAP, 2); break;
    case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8:
    case 0xc7: case 0xc8: case 0xc9:
      throw Error("msgpack: ext types are not part of the Janus packet schema");
    default:  // 0xc1 (never used)
      throw Error("msgpack: invalid type byte 0xc1");
  }
}

}  // namespace
}  // namespace janus

using namespace janus;

extern "C" int janus_pack_packet(const janus_packet* pkt, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    JANUS_CHECK(pkt && out_len, "null argument");
    Out o{out, cap};
    // Insertion order of JanusPacket.to_dict (protocol.py:67-74): t, m, p, ts[, o].
    const bool has_o = pkt->override_emotion != nullptr;
    pack_map_header(o, has_o ? 5 : 4);
    pack_str(o, "t", 1);
    pack_str(o, pkt->text, pkt->text_len);
    pack_str(o, "m", 1);
    pack_int(o, pkt->mode);
    pack_str(o, "p", 1);
    pack_map_header(o, (size_t)pkt->n_prosody);
    for (int k = 0; k < pkt->n_prosody; ++k) {
      pack_str(o, pkt->prosody_keys[k].s, pkt->prosody_keys[k].len);
      pack_value(o, pkt->prosody_vals[k]);
    }
    pack_str(o, "ts", 2);
    pack_value(o, pkt->timestamp);
    if (has_o) {
      pack_str(o, "o", 1);
      pack_str(o, pkt->override_emotion, pkt->override_len);
    }
    *out_len = o.n;
    JANUS_CHECK(!o.overflow, "output buffer too small (need " + std::to_string(o.n) + " bytes)");
  });
}

extern "C" int janus_unpack(const uint8_t* buf, size_t len, janus_mp_node* nodes, size_t cap,
                            size_t* n_nodes) {
  return guarded([&] {
    JANUS_CHECK(buf || len == 0, "null buffer");
    JANUS_CHECK(nodes && n_nodes, "null argument");
    In in{buf, len};
    Nodes nd{nodes, cap};
    decode(in, nd, 0);
    JANUS_CHECK(in.pos == len, "msgpack: extra data after the packet (" +
                                   std::to_string(len - in.pos) + " bytes)");
    *n_nodes = nd.n;
  });
}
