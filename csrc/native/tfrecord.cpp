// TFRecord framing for TensorBoard event files (the reference's Keras TensorBoard callback,
// /root/reference/client_fit_model.py:153-154, writes tfevents; TensorFlow is not available here).
// Record = uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data), little endian.
// CRC32C (Castagnoli, reflected polynomial 0x82F63B78), slicing-by-8 tables.
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace py = pybind11;

namespace tfrec {

static uint32_t T[8][256];
static bool init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    T[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int s = 1; s < 8; ++s) T[s][i] = (T[s - 1][i] >> 8) ^ T[0][T[s - 1][i] & 0xff];
  return true;
}
static const bool kInit = init_tables();

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0) {
  (void)kInit;
  crc = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= crc;
    crc = T[7][v & 0xff] ^ T[6][(v >> 8) & 0xff] ^ T[5][(v >> 16) & 0xff] ^ T[4][(v >> 24) & 0xff] ^
          T[3][(v >> 32) & 0xff] ^ T[2][(v >> 40) & 0xff] ^ T[1][(v >> 48) & 0xff] ^ T[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ T[0][(crc ^ *p++) & 0xff];
  return ~crc;
}

uint32_t masked(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

py::bytes frame(py::bytes data) {
  std::string d = data;
  const uint64_t len = d.size();
  std::string out(8 + 4 + d.size() + 4, '\0');
  std::memcpy(&out[0], &len, 8);
  const uint32_t lc = masked(crc32c(reinterpret_cast<const uint8_t*>(&len), 8));
  std::memcpy(&out[8], &lc, 4);
  std::memcpy(&out[12], d.data(), d.size());
  const uint32_t dc = masked(crc32c(reinterpret_cast<const uint8_t*>(d.data()), d.size()));
  std::memcpy(&out[12 + d.size()], &dc, 4);
  return py::bytes(out);
}

// split a TFRecord stream into records, verifying both checksums
py::list unframe(py::bytes stream) {
  std::string s = stream;
  py::list out;
  size_t off = 0;
  while (off < s.size()) {
    if (off + 12 > s.size()) throw std::runtime_error("tfrecord: truncated header");
    uint64_t len;
    uint32_t lc, dc;
    std::memcpy(&len, &s[off], 8);
    std::memcpy(&lc, &s[off + 8], 4);
    if (masked(crc32c(reinterpret_cast<const uint8_t*>(&s[off]), 8)) != lc)
      throw std::runtime_error("tfrecord: bad length crc");
    if (off + 12 + len + 4 > s.size()) throw std::runtime_error("tfrecord: truncated record");
    std::memcpy(&dc, &s[off + 12 + len], 4);
    if (masked(crc32c(reinterpret_cast<const uint8_t*>(&s[off + 12]), len)) != dc)
      throw std::runtime_error("tfrecord: bad data crc");
    out.append(py::bytes(s.data() + off + 12, len));
    off += 12 + len + 4;
  }
  return out;
}

}  // namespace tfrec

void register_tfrecord(py::module_& m) {
  auto t = m.def_submodule("tfrecord", "TFRecord framing (masked CRC32C)");
  t.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return tfrec::crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  t.def("frame", &tfrec::frame);
  t.def("unframe", &tfrec::unframe);
}
