// _native: host-side C++ components of the framework (no GPU needed).
//   h5lite   - Keras-layout HDF5 writer/reader            (csrc/native/h5lite.cpp)
//   contour  - crack contour geometry (cv2 subset)          (csrc/native/contour.cpp)
//   imgproc  - cv2.resize(INTER_LINEAR)-style bilinear resize + mask binarisation used by the folder loader
//              (reference: cv2.imread/cvtColor/resize, /root/reference/client_fit_model.py:34-40)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

namespace py = pybind11;
void register_h5lite(py::module_& m);
void register_contour(py::module_& m);

namespace imgproc {
// Half-pixel-centre bilinear resize with border clamping (the INTER_LINEAR sampling grid of cv2.resize).
static void resize_rows(const uint8_t* src, int sh, int sw, int c, uint8_t* dst, int dh, int dw, int r0, int r1) {
  const float fy = (float)sh / dh, fx = (float)sw / dw;
  std::vector<int> x0(dw), x1(dw);
  std::vector<float> ax(dw);
  for (int x = 0; x < dw; ++x) {
    float sx = (x + 0.5f) * fx - 0.5f;
    int ix = (int)std::floor(sx);
    float a = sx - ix;
    if (ix < 0) { ix = 0; a = 0.f; }
    if (ix >= sw - 1) { ix = sw - 1; a = 0.f; }
    x0[x] = ix; x1[x] = std::min(ix + 1, sw - 1); ax[x] = a;
  }
  for (int y = r0; y < r1; ++y) {
    float sy = (y + 0.5f) * fy - 0.5f;
    int iy = (int)std::floor(sy);
    float b = sy - iy;
    if (iy < 0) { iy = 0; b = 0.f; }
    if (iy >= sh - 1) { iy = sh - 1; b = 0.f; }
    int iy1 = std::min(iy + 1, sh - 1);
    const uint8_t* ra = src + (size_t)iy * sw * c;
    const uint8_t* rb = src + (size_t)iy1 * sw * c;
    uint8_t* o = dst + (size_t)y * dw * c;
    for (int x = 0; x < dw; ++x)
      for (int k = 0; k < c; ++k) {
        float t = ra[x0[x] * c + k] * (1 - ax[x]) + ra[x1[x] * c + k] * ax[x];
        float u = rb[x0[x] * c + k] * (1 - ax[x]) + rb[x1[x] * c + k] * ax[x];
        float v = t * (1 - b) + u * b;
        o[x * c + k] = (uint8_t)std::min(255.f, std::max(0.f, std::nearbyint(v)));
      }
  }
}

py::array_t<uint8_t> resize(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img, int dh, int dw, int threads) {
  if (img.ndim() != 2 && img.ndim() != 3) throw std::runtime_error("resize expects HxW or HxWxC uint8");
  int sh = (int)img.shape(0), sw = (int)img.shape(1), c = img.ndim() == 3 ? (int)img.shape(2) : 1;
  std::vector<py::ssize_t> shape = {dh, dw};
  if (img.ndim() == 3) shape.push_back(c);
  py::array_t<uint8_t> out(shape);
  const uint8_t* s = img.data();
  uint8_t* d = out.mutable_data();
  {
    py::gil_scoped_release rel;
    int T = std::max(1, std::min(threads, dh));
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t) ts.emplace_back(resize_rows, s, sh, sw, c, d, dh, dw, dh * t / T, dh * (t + 1) / T);
    for (auto& th : ts) th.join();
  }
  return out;
}
}  // namespace imgproc

void register_tfrecord(py::module_& m);

PYBIND11_MODULE(_native, m) {
  m.doc() = "host-side native components (HDF5, contours, image resize, TFRecord framing)";
  register_h5lite(m);
  register_contour(m);
  register_tfrecord(m);
  m.def("resize_bilinear", &imgproc::resize, py::arg("img"), py::arg("height"), py::arg("width"), py::arg("threads") = 4);
}
