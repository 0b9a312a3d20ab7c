// Minimal HDF5 writer/reader for Keras-layout checkpoints.
//
// The reference saves Keras full-model HDF5 via h5py/libhdf5 (ModelCheckpoint("crack_segmentation.h5"),
// /root/reference/test/Segmentation.py:177-178; layout SURVEY.md §5.4). Neither h5py nor libhdf5 is available to the
// framework, so this implements the subset Keras files use, in the "earliest" library format that h5py writes:
//   superblock v0, version-1 object headers (+ continuation messages on read), symbol-table groups
//   (v1 B-tree + local heap + symbol-table nodes), attributes (message v1 written; v1-v3 read), datatypes
//   fixed-point / IEEE float / fixed-length string (+ variable-length string via global heap on read),
//   simple/scalar dataspaces, contiguous + compact layouts. Chunked/filtered datasets are rejected on read.
//
// Data model exchanged with Python (pybind11): a node is a dict
//   {"attrs": {name: value}, "groups": {name: node}, "datasets": {name: {"data": ndarray, "attrs": {...}}}}
// attribute values: str (fixed-length string scalar), list[str|bytes] (fixed-length string array),
// or ndarray/number (float32/float64/int32/int64).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace h5lite {

static const uint64_t UNDEF = ~0ull;
static const int LEAF_K = 4;       // group leaf node K  -> 2K = 8 entries per symbol-table node
static const int INTERNAL_K = 16;  // group internal node K -> 2K = 32 children per B-tree node

// ------------------------------------------------------------------------------------------------------------
// in-memory tree
enum class DKind { F32, F64, I32, I64, U8, STR };

struct Value {
  DKind kind = DKind::F32;
  std::vector<uint64_t> shape;     // empty = scalar
  std::vector<uint8_t> bytes;      // raw little-endian payload (STR: elements of `strsize` bytes, null padded)
  size_t strsize = 0;
  size_t elem_size() const {
    switch (kind) {
      case DKind::F32: case DKind::I32: return 4;
      case DKind::F64: case DKind::I64: return 8;
      case DKind::U8: return 1;
      case DKind::STR: return strsize;
    }
    return 1;
  }
};

struct Node;
struct Dataset {
  Value value;
  std::vector<std::pair<std::string, Value>> attrs;
};
struct Node {
  std::vector<std::pair<std::string, Value>> attrs;
  std::map<std::string, std::unique_ptr<Node>> groups;      // std::map keeps names strcmp-sorted
  std::map<std::string, std::unique_ptr<Dataset>> datasets;
};

// ------------------------------------------------------------------------------------------------------------
// writer
class Buf {
 public:
  std::vector<uint8_t> d;
  size_t size() const { return d.size(); }
  void u8(uint8_t v) { d.push_back(v); }
  void u16(uint16_t v) { for (int i = 0; i < 2; ++i) d.push_back((v >> (8 * i)) & 0xff); }
  void u32(uint32_t v) { for (int i = 0; i < 4; ++i) d.push_back((v >> (8 * i)) & 0xff); }
  void u64(uint64_t v) { for (int i = 0; i < 8; ++i) d.push_back((v >> (8 * i)) & 0xff); }
  void raw(const void* p, size_t n) { const uint8_t* b = (const uint8_t*)p; d.insert(d.end(), b, b + n); }
  void zeros(size_t n) { d.insert(d.end(), n, 0); }
  void pad8() { while (d.size() % 8) d.push_back(0); }
  void put_u64(size_t at, uint64_t v) { for (int i = 0; i < 8; ++i) d[at + i] = (v >> (8 * i)) & 0xff; }
  void put_u32(size_t at, uint32_t v) { for (int i = 0; i < 4; ++i) d[at + i] = (v >> (8 * i)) & 0xff; }
};

static size_t pad8(size_t n) { return (n + 7) / 8 * 8; }

static void enc_datatype(Buf& b, const Value& v) {
  switch (v.kind) {
    case DKind::F32:
      b.u8(0x11); b.u8(0x20); b.u8(31); b.u8(0); b.u32(4);
      b.u16(0); b.u16(32); b.u8(23); b.u8(8); b.u8(0); b.u8(23); b.u32(127);
      break;
    case DKind::F64:
      b.u8(0x11); b.u8(0x20); b.u8(63); b.u8(0); b.u32(8);
      b.u16(0); b.u16(64); b.u8(52); b.u8(11); b.u8(0); b.u8(52); b.u32(1023);
      break;
    case DKind::I32: b.u8(0x10); b.u8(0x08); b.u8(0); b.u8(0); b.u32(4); b.u16(0); b.u16(32); break;
    case DKind::I64: b.u8(0x10); b.u8(0x08); b.u8(0); b.u8(0); b.u32(8); b.u16(0); b.u16(64); break;
    case DKind::U8: b.u8(0x10); b.u8(0x00); b.u8(0); b.u8(0); b.u32(1); b.u16(0); b.u16(8); break;
    case DKind::STR:  // fixed-length, null padded, ASCII (what h5py writes for numpy 'S' arrays)
      b.u8(0x13); b.u8(0x01); b.u8(0); b.u8(0); b.u32((uint32_t)v.strsize);
      break;
  }
}

static void enc_dataspace(Buf& b, const Value& v) {
  b.u8(1); b.u8((uint8_t)v.shape.size()); b.u8(0); b.u8(0); b.u32(0);
  for (auto s : v.shape) b.u64(s);
}

struct Msg { uint16_t type; std::vector<uint8_t> data; };

static Msg attr_msg(const std::string& name, const Value& v) {
  Buf dt, ds;
  enc_datatype(dt, v);
  enc_dataspace(ds, v);
  Buf m;
  m.u8(1); m.u8(0);
  m.u16((uint16_t)(name.size() + 1)); m.u16((uint16_t)dt.size()); m.u16((uint16_t)ds.size());
  m.raw(name.data(), name.size()); m.u8(0); m.pad8();
  m.raw(dt.d.data(), dt.size()); m.pad8();
  m.raw(ds.d.data(), ds.size()); m.pad8();
  m.raw(v.bytes.data(), v.bytes.size());
  if (m.size() > 65000) throw std::runtime_error("attribute '" + name + "' exceeds the 64 KiB header message limit");
  return {0x000C, m.d};
}

class Writer {
 public:
  Buf f;
  // returns the address of the object header
  uint64_t obj_header(const std::vector<Msg>& msgs) {
    f.pad8();
    uint64_t addr = f.size();
    size_t body = 0;
    for (auto& m : msgs) body += 8 + pad8(m.data.size());
    f.u8(1); f.u8(0); f.u16((uint16_t)msgs.size()); f.u32(1); f.u32((uint32_t)body); f.u32(0);  // 16-byte prefix
    for (auto& m : msgs) {
      f.u16(m.type); f.u16((uint16_t)pad8(m.data.size())); f.u8(0); f.zeros(3);
      f.raw(m.data.data(), m.data.size());
      f.pad8();
    }
    return addr;
  }

  uint64_t dataset(const Dataset& ds) {
    f.pad8();
    uint64_t data_addr = f.size();
    f.raw(ds.value.bytes.data(), ds.value.bytes.size());
    std::vector<Msg> msgs;
    { Buf b; enc_dataspace(b, ds.value); msgs.push_back({0x0001, b.d}); }
    { Buf b; enc_datatype(b, ds.value); msgs.push_back({0x0003, b.d}); }
    { Buf b; b.u8(2); b.u8(2); b.u8(2); b.u8(0); msgs.push_back({0x0005, b.d}); }   // fill value v2: none
    { Buf b; b.u8(3); b.u8(1); b.u64(ds.value.bytes.empty() ? UNDEF : data_addr); b.u64(ds.value.bytes.size());
      msgs.push_back({0x0008, b.d}); }                                                 // contiguous layout v3
    for (auto& a : ds.attrs) msgs.push_back(attr_msg(a.first, a.second));
    return obj_header(msgs);
  }

  struct GroupAddrs { uint64_t ohdr, btree, heap; };

  GroupAddrs group(const Node& n) {
    // children first (their addresses go into the symbol-table nodes)
    struct Child { std::string name; uint64_t ohdr; bool is_group; uint64_t btree, heap; };
    std::vector<Child> kids;
    for (auto& g : n.groups) { auto a = group(*g.second); kids.push_back({g.first, a.ohdr, true, a.btree, a.heap}); }
    for (auto& d : n.datasets) kids.push_back({d.first, dataset(*d.second), false, 0, 0});
    std::sort(kids.begin(), kids.end(), [](const Child& a, const Child& b) { return a.name < b.name; });
    // local heap: "" at offset 0, then names (null terminated, 8-aligned)
    Buf heap;
    heap.zeros(8);
    std::vector<uint64_t> name_off;
    for (auto& k : kids) { name_off.push_back(heap.size()); heap.raw(k.name.data(), k.name.size()); heap.u8(0); heap.pad8(); }
    // trailing free block (16 bytes) so the heap has a well-formed free list
    uint64_t free_off = heap.size();
    heap.u64(1); heap.u64(16);
    f.pad8();
    uint64_t heap_addr = f.size();
    f.raw("HEAP", 4); f.u8(0); f.zeros(3); f.u64(heap.size()); f.u64(free_off); f.u64(heap_addr + 32);
    f.raw(heap.d.data(), heap.size());
    // symbol-table nodes, 2*LEAF_K entries each
    const size_t per = 2 * LEAF_K;
    size_t nnodes = kids.empty() ? 1 : (kids.size() + per - 1) / per;
    if (nnodes > (size_t)2 * INTERNAL_K) throw std::runtime_error("group too large for a single-level B-tree");
    std::vector<uint64_t> snod_addr;
    std::vector<uint64_t> last_name;
    for (size_t s = 0; s < nnodes; ++s) {
      f.pad8();
      snod_addr.push_back(f.size());
      size_t lo = s * per, hi = std::min(kids.size(), lo + per);
      f.raw("SNOD", 4); f.u8(1); f.u8(0); f.u16((uint16_t)(hi - lo));
      for (size_t i = 0; i < per; ++i) {
        if (lo + i < hi) {
          const Child& k = kids[lo + i];
          f.u64(name_off[lo + i]); f.u64(k.ohdr);
          if (k.is_group) { f.u32(1); f.u32(0); f.u64(k.btree); f.u64(k.heap); }
          else { f.u32(0); f.u32(0); f.zeros(16); }
        } else {
          f.zeros(40);
        }
      }
      last_name.push_back(hi > lo ? name_off[hi - 1] : 0);
    }
    // v1 B-tree (type 0 = group), single leaf level; node sized for 2K children / 2K+1 keys
    f.pad8();
    uint64_t btree_addr = f.size();
    uint16_t used = kids.empty() ? 0 : (uint16_t)nnodes;
    f.raw("TREE", 4); f.u8(0); f.u8(0); f.u16(used); f.u64(UNDEF); f.u64(UNDEF);
    for (int i = 0; i < 2 * INTERNAL_K; ++i) {
      f.u64(i == 0 ? 0 : (i - 1 < (int)last_name.size() ? last_name[i - 1] : 0));   // key i
      f.u64(i < (int)used ? snod_addr[i] : 0);                                           // child i
    }
    f.u64(used ? last_name[used - 1] : 0);                                               // key 2K
    std::vector<Msg> msgs;
    { Buf b; b.u64(btree_addr); b.u64(heap_addr); msgs.push_back({0x0011, b.d}); }
    for (auto& a : n.attrs) msgs.push_back(attr_msg(a.first, a.second));
    uint64_t oh = obj_header(msgs);
    return {oh, btree_addr, heap_addr};
  }

  std::vector<uint8_t> write(const Node& root) {
    f.d.assign(96, 0);   // superblock v0 placeholder
    auto r = group(root);
    f.pad8();
    uint64_t eof = f.size();
    Buf sb;
    const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
    sb.raw(sig, 8);
    sb.u8(0); sb.u8(0); sb.u8(0); sb.u8(0);
    sb.u8(0); sb.u8(8); sb.u8(8); sb.u8(0);
    sb.u16(LEAF_K); sb.u16(INTERNAL_K);
    sb.u32(0);
    sb.u64(0); sb.u64(UNDEF); sb.u64(eof); sb.u64(UNDEF);
    sb.u64(0); sb.u64(r.ohdr); sb.u32(1); sb.u32(0); sb.u64(r.btree); sb.u64(r.heap);
    std::memcpy(f.d.data(), sb.d.data(), 96);
    return f.d;
  }
};

// ------------------------------------------------------------------------------------------------------------
// reader
class Reader {
 public:
  std::vector<uint8_t> d;
  int so = 8, sl = 8;  // size of offsets / lengths
  explicit Reader(std::vector<uint8_t> data) : d(std::move(data)) {}

  void need(uint64_t at, uint64_t n) const {
    if (at > d.size() || n > d.size() - at) throw std::runtime_error("h5lite: truncated or corrupt file");
  }
  uint64_t un(uint64_t at, int n) const {
    need(at, n);
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v |= (uint64_t)d[at + i] << (8 * i);
    return v;
  }
  uint64_t off(uint64_t at) const { return un(at, so); }
  uint64_t len(uint64_t at) const { return un(at, sl); }

  struct Dtype { int cls = -1; size_t size = 0; bool sign = false; bool be = false; bool vlen_str = false; };
  struct Space { std::vector<uint64_t> dims; };

  Dtype parse_dtype(uint64_t at) const {
    Dtype t;
    uint8_t cv = (uint8_t)un(at, 1);
    t.cls = cv & 0x0f;
    uint32_t bits = (uint32_t)un(at + 1, 3);
    t.size = (size_t)un(at + 4, 4);
    if (t.cls == 0) { t.be = bits & 1; t.sign = bits & 8; }
    else if (t.cls == 1) { t.be = bits & 1; }
    else if (t.cls == 9) { t.vlen_str = ((bits & 0xf) == 1); }
    return t;
  }

  Space parse_space(uint64_t at) const {
    Space s;
    int ver = (int)un(at, 1), rank = (int)un(at + 1, 1), flags = (int)un(at + 2, 1);
    uint64_t p;
    if (ver == 1) p = at + 8;
    else if (ver == 2) { p = at + 4; if ((int)un(at + 3, 1) == 2) rank = 0; }
    else throw std::runtime_error("h5lite: unsupported dataspace version");
    (void)flags;
    for (int i = 0; i < rank; ++i) s.dims.push_back(len(p + (uint64_t)i * sl));
    return s;
  }

  std::string read_vlen_str(uint64_t at) const {   // 4-byte length, then global heap id (collection addr, index)
    uint32_t n = (uint32_t)un(at, 4);
    uint64_t coll = off(at + 4);
    uint32_t idx = (uint32_t)un(at + 4 + so, 4);
    if (n == 0 || coll == UNDEF) return std::string();
    need(coll, 16);
    if (std::memcmp(&d[coll], "GCOL", 4) != 0) throw std::runtime_error("h5lite: bad global heap");
    uint64_t csize = len(coll + 8);
    uint64_t p = coll + 8 + sl;
    uint64_t end = coll + csize;
    while (p + 8 + sl <= end) {
      uint16_t oi = (uint16_t)un(p, 2);
      uint64_t osz = len(p + 8);
      if (oi == 0) break;
      if (oi == idx) { need(p + 8 + sl, osz); return std::string((const char*)&d[p + 8 + sl], std::min<uint64_t>(osz, n)); }
      p += 8 + sl + pad8(osz);
    }
    throw std::runtime_error("h5lite: global heap object not found");
  }

  py::object make_value(const Dtype& t, const Space& s, uint64_t data_at) const {
    uint64_t count = 1;
    for (auto x : s.dims) count *= x;
    std::vector<py::ssize_t> shape(s.dims.begin(), s.dims.end());
    if (t.cls == 3 || (t.cls == 9 && t.vlen_str)) {
      py::list out;
      for (uint64_t i = 0; i < count; ++i) {
        std::string str;
        if (t.cls == 3) {
          need(data_at + i * t.size, t.size);
          const char* p = (const char*)&d[data_at + i * t.size];
          size_t n = strnlen(p, t.size);
          str.assign(p, n);
        } else {
          str = read_vlen_str(data_at + i * (4 + so + 4));
        }
        out.append(py::bytes(str));
      }
      if (s.dims.empty()) return out[0];
      return out;
    }
    std::string fmt;
    if (t.cls == 1) fmt = t.size == 4 ? "<f4" : t.size == 8 ? "<f8" : "";
    else if (t.cls == 0) fmt = std::string(t.sign ? "<i" : "<u") + std::to_string(t.size);
    if (fmt.empty()) throw std::runtime_error("h5lite: unsupported datatype class " + std::to_string(t.cls));
    if (t.be) fmt[0] = '>';
    need(data_at, count * t.size);
    py::array arr(py::dtype(fmt), shape);
    std::memcpy(arr.mutable_data(), &d[data_at], count * t.size);
    return arr;
  }

  struct Obj {
    std::vector<std::pair<uint16_t, std::pair<uint64_t, uint64_t>>> msgs;  // type -> (data addr, size)
  };

  Obj read_ohdr(uint64_t at) const {
    Obj o;
    need(at, 16);
    if (std::memcmp(&d[at], "OHDR", 4) == 0) return read_ohdr_v2(at);
    if (un(at, 1) != 1) throw std::runtime_error("h5lite: unsupported object header version");
    int nmsg = (int)un(at + 2, 2);
    uint64_t size = un(at + 8, 4);
    std::vector<std::pair<uint64_t, uint64_t>> blocks = {{at + 16, size}};
    int seen = 0;
    for (size_t bi = 0; bi < blocks.size() && seen < nmsg; ++bi) {
      uint64_t p = blocks[bi].first, end = blocks[bi].first + blocks[bi].second;
      while (p + 8 <= end && seen < nmsg) {
        uint16_t type = (uint16_t)un(p, 2);
        uint64_t msz = un(p + 2, 2);
        if (type == 0x0010) blocks.push_back({off(p + 8), len(p + 8 + so)});
        else o.msgs.push_back({type, {p + 8, msz}});
        p += 8 + msz;
        ++seen;
      }
    }
    return o;
  }

  Obj read_ohdr_v2(uint64_t at) const {
    Obj o;
    int flags = (int)un(at + 5, 1);
    uint64_t p = at + 6;
    if (flags & 0x20) p += 16;
    if (flags & 0x10) p += 4;
    int szb = 1 << (flags & 3);
    uint64_t csize = un(p, szb);
    p += szb;
    std::vector<std::pair<uint64_t, uint64_t>> blocks = {{p, csize}};
    for (size_t bi = 0; bi < blocks.size(); ++bi) {
      uint64_t q = blocks[bi].first, end = blocks[bi].first + blocks[bi].second;
      if (bi > 0) q += 4;  // "OCHK"
      while (q + 4 + ((flags & 4) ? 2 : 0) <= end) {
        uint16_t type = (uint16_t)un(q, 1);
        uint64_t msz = un(q + 1, 2);
        uint64_t hdr = 4 + ((flags & 4) ? 2 : 0);
        if (type == 0x0010) blocks.push_back({off(q + hdr), len(q + hdr + so)});
        else if (type != 0) o.msgs.push_back({type, {q + hdr, msz}});
        q += hdr + msz;
      }
    }
    return o;
  }

  py::tuple parse_attr(uint64_t at) const {
    int ver = (int)un(at, 1);
    uint64_t nsz = un(at + 2, 2), tsz = un(at + 4, 2), ssz = un(at + 6, 2);
    uint64_t p = at + 8;
    if (ver == 3) p += 1;
    std::string name((const char*)&d[p], strnlen((const char*)&d[p], nsz));
    if (ver == 1) { p += pad8(nsz); } else p += nsz;
    uint64_t tp = p;
    p += (ver == 1) ? pad8(tsz) : tsz;
    uint64_t sp = p;
    p += (ver == 1) ? pad8(ssz) : ssz;
    return py::make_tuple(name, make_value(parse_dtype(tp), parse_space(sp), p));
  }

  void collect_symtab(uint64_t btree, uint64_t heap_addr, std::vector<std::pair<std::string, uint64_t>>& out) const {
    need(btree, 24);
    if (std::memcmp(&d[btree], "TREE", 4) != 0) throw std::runtime_error("h5lite: bad B-tree node");
    int level = (int)un(btree + 5, 1);
    int used = (int)un(btree + 6, 2);
    uint64_t heap_data = off(heap_addr + 8 + 2 * sl);
    uint64_t p = btree + 8 + 2 * so;
    for (int i = 0; i < used; ++i) {
      uint64_t child = off(p + sl + (uint64_t)i * (sl + so));
      if (level > 0) { collect_symtab(child, heap_addr, out); continue; }
      need(child, 8);
      if (std::memcmp(&d[child], "SNOD", 4) != 0) throw std::runtime_error("h5lite: bad symbol-table node");
      int n = (int)un(child + 6, 2);
      uint64_t e = child + 8;
      for (int k = 0; k < n; ++k, e += so + so + 4 + 4 + 16) {
        uint64_t noff = off(e);
        const char* nm = (const char*)&d[heap_data + noff];
        out.push_back({std::string(nm), off(e + so)});
      }
    }
  }

  py::dict read_object(uint64_t at, int depth) const {
    if (depth > 64) throw std::runtime_error("h5lite: object nesting too deep");
    Obj o = read_ohdr(at);
    py::dict attrs, groups, datasets, out;
    bool is_group = false;
    Dtype dt; Space sp; bool have_dt = false, have_sp = false;
    int layout_cls = -1; uint64_t data_addr = UNDEF, data_size = 0, compact_at = 0;
    std::vector<std::pair<std::string, uint64_t>> links;
    for (auto& m : o.msgs) {
      uint16_t type = m.first;
      uint64_t p = m.second.first;
      if (type == 0x000C) { auto t = parse_attr(p); attrs[t[0]] = t[1]; }
      else if (type == 0x0011) { is_group = true; collect_symtab(off(p), off(p + so), links); }
      else if (type == 0x0006) {   // link message (new-style compact groups)
        is_group = true;
        int flags = (int)un(p + 1, 1);
        uint64_t q = p + 2;
        int ltype = 0;
        if (flags & 0x8) { ltype = (int)un(q, 1); q += 1; }
        if (flags & 0x4) q += 8;
        if (flags & 0x10) q += 1;
        int lsz = 1 << (flags & 3);
        uint64_t nl = un(q, lsz); q += lsz;
        std::string name((const char*)&d[q], nl); q += nl;
        if (ltype == 0) links.push_back({name, off(q)});
      }
      else if (type == 0x0003) { dt = parse_dtype(p); have_dt = true; }
      else if (type == 0x0001) { sp = parse_space(p); have_sp = true; }
      else if (type == 0x0008) {
        int ver = (int)un(p, 1);
        if (ver < 3) throw std::runtime_error("h5lite: unsupported layout message version");
        layout_cls = (int)un(p + 1, 1);
        if (layout_cls == 1) { data_addr = off(p + 2); data_size = len(p + 2 + so); }
        else if (layout_cls == 0) { data_size = un(p + 2, 2); compact_at = p + 4; }
      }
      else if (type == 0x000B) throw std::runtime_error("h5lite: filtered (compressed) datasets are not supported");
    }
    for (auto& l : links) {
      py::dict child = read_object(l.second, depth + 1);
      if (child.contains("datasets") || child.contains("groups")) groups[py::str(l.first)] = child;
      else datasets[py::str(l.first)] = child;
    }
    if (is_group || (!have_dt && !have_sp)) {
      out["attrs"] = attrs; out["groups"] = groups; out["datasets"] = datasets;
      return out;
    }
    if (!have_dt || !have_sp) throw std::runtime_error("h5lite: dataset without datatype/dataspace");
    if (layout_cls == 2) throw std::runtime_error("h5lite: chunked datasets are not supported");
    uint64_t at_data = layout_cls == 0 ? compact_at : data_addr;
    py::object val;
    uint64_t count = 1;
    for (auto x : sp.dims) count *= x;
    if (at_data == UNDEF || (layout_cls == 1 && data_size == 0 && count > 0)) {
      // never written: zeros
      Value z;
      std::vector<uint8_t> zeros(count * std::max<size_t>(dt.size, 1), 0);
      Reader zr(zeros);
      val = zr.make_value(dt, sp, 0);
    } else {
      val = make_value(dt, sp, at_data);
    }
    out["data"] = val;
    out["attrs"] = attrs;
    return out;
  }

  py::dict read() {
    need(0, 8);
    const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
    uint64_t base = 0;
    while (base + 8 <= d.size() && std::memcmp(&d[base], sig, 8) != 0) {   // user block: 512, 1024, ...
      base = base ? base * 2 : 512;
      if (base > d.size()) throw std::runtime_error("h5lite: not an HDF5 file");
    }
    int ver = (int)un(base + 8, 1);
    uint64_t root;
    if (ver == 0 || ver == 1) {
      so = (int)un(base + 13, 1); sl = (int)un(base + 14, 1);
      uint64_t p = base + 24 + (ver == 1 ? 4 : 0);
      p += 4 * (uint64_t)so;              // base, free-space, eof, driver
      root = off(p + so);                 // symbol table entry: name offset, header address
    } else if (ver == 2 || ver == 3) {
      so = (int)un(base + 9, 1); sl = (int)un(base + 10, 1);
      root = off(base + 12 + 3 * (uint64_t)so);
    } else {
      throw std::runtime_error("h5lite: unsupported superblock version");
    }
    if (base) {
      // addresses are relative to the base address; simplest: drop the user block
      d.erase(d.begin(), d.begin() + (long)base);
    }
    return read_object(root, 0);
  }
};

// ------------------------------------------------------------------------------------------------------------
// python conversion
static Value to_value(py::handle h) {
  Value v;
  if (py::isinstance<py::str>(h) || py::isinstance<py::bytes>(h)) {
    std::string s = py::isinstance<py::str>(h) ? h.cast<std::string>() : std::string(h.cast<py::bytes>());
    v.kind = DKind::STR;
    v.strsize = std::max<size_t>(s.size(), 1);
    v.bytes.assign(v.strsize, 0);
    std::memcpy(v.bytes.data(), s.data(), s.size());
    return v;
  }
  if (py::isinstance<py::list>(h) || py::isinstance<py::tuple>(h)) {
    std::vector<std::string> items;
    for (auto it : h) items.push_back(py::isinstance<py::str>(it) ? it.cast<std::string>()
                                                                  : std::string(it.cast<py::bytes>()));
    size_t mx = 1;
    for (auto& s : items) mx = std::max(mx, s.size());
    v.kind = DKind::STR;
    v.strsize = mx;
    v.shape = {items.size()};
    v.bytes.assign(items.size() * mx, 0);
    for (size_t i = 0; i < items.size(); ++i) std::memcpy(&v.bytes[i * mx], items[i].data(), items[i].size());
    return v;
  }
  py::array arr = py::array::ensure(h);
  if (!arr) throw std::runtime_error("h5lite: unsupported attribute/dataset value");
  char k = arr.dtype().kind();
  size_t isz = arr.dtype().itemsize();
  if (k == 'f' && isz == 4) v.kind = DKind::F32;
  else if (k == 'f' && isz == 8) v.kind = DKind::F64;
  else if (k == 'i' && isz == 4) v.kind = DKind::I32;
  else if (k == 'i' && isz == 8) v.kind = DKind::I64;
  else if (k == 'u' && isz == 1) v.kind = DKind::U8;
  else throw std::runtime_error("h5lite: unsupported dtype");
  py::array c = py::array::ensure(arr, py::array::c_style | py::array::forcecast);
  for (py::ssize_t i = 0; i < c.ndim(); ++i) v.shape.push_back((uint64_t)c.shape(i));
  v.bytes.resize((size_t)c.nbytes());
  std::memcpy(v.bytes.data(), c.data(), (size_t)c.nbytes());
  return v;
}

static std::unique_ptr<Node> to_node(py::dict n) {
  auto node = std::make_unique<Node>();
  if (n.contains("attrs"))
    for (auto kv : n["attrs"].cast<py::dict>()) node->attrs.push_back({kv.first.cast<std::string>(), to_value(kv.second)});
  if (n.contains("groups"))
    for (auto kv : n["groups"].cast<py::dict>()) node->groups[kv.first.cast<std::string>()] = to_node(kv.second.cast<py::dict>());
  if (n.contains("datasets"))
    for (auto kv : n["datasets"].cast<py::dict>()) {
      auto ds = std::make_unique<Dataset>();
      py::object o = py::reinterpret_borrow<py::object>(kv.second);
      if (py::isinstance<py::dict>(o)) {
        py::dict dd = o.cast<py::dict>();
        ds->value = to_value(dd["data"]);
        if (dd.contains("attrs"))
          for (auto a : dd["attrs"].cast<py::dict>()) ds->attrs.push_back({a.first.cast<std::string>(), to_value(a.second)});
      } else {
        ds->value = to_value(o);
      }
      node->datasets[kv.first.cast<std::string>()] = std::move(ds);
    }
  return node;
}

py::bytes write_bytes(py::dict tree) {
  auto root = to_node(tree);
  Writer w;
  auto out = w.write(*root);
  return py::bytes((const char*)out.data(), out.size());
}

void write_file(const std::string& path, py::dict tree) {
  auto root = to_node(tree);
  Writer w;
  auto out = w.write(*root);
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("h5lite: cannot open " + path);
  f.write((const char*)out.data(), (std::streamsize)out.size());
}

py::dict read_bytes(py::bytes b) {
  std::string s = b;
  Reader r(std::vector<uint8_t>(s.begin(), s.end()));
  return r.read();
}

py::dict read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("h5lite: cannot open " + path);
  std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  Reader r(std::move(data));
  return r.read();
}

}  // namespace h5lite

void register_h5lite(py::module_& m) {
  auto h = m.def_submodule("h5lite", "minimal HDF5 (Keras layout) writer/reader");
  h.def("write_bytes", &h5lite::write_bytes);
  h.def("write_file", &h5lite::write_file);
  h.def("read_bytes", &h5lite::read_bytes);
  h.def("read_file", &h5lite::read_file);
}
