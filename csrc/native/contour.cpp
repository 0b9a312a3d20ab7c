// Crack contour analysis: the OpenCV calls of the reference's post-processing, natively.
//
// Reference (/root/reference/test/Segmentation2.py:114-141, called from client_fit_model.py:215):
//   cvtColor(BGR2GRAY) -> threshold(127, 255, BINARY) -> findContours(RETR_TREE, CHAIN_APPROX_SIMPLE)
//   -> contourArea(contours[0]), arcLength(contours[0], closed) , approxPolyDP(eps = 0.01 / 0.1 * perimeter)
// cv2 is not installed, so this implements Suzuki & Abe (1985) border following (8-connected foreground, full
// hierarchy as RETR_TREE), chain compression (CHAIN_APPROX_SIMPLE), the shoelace area, closed arc length and
// Douglas-Peucker polygon approximation. Contour order follows the raster discovery order; OpenCV's exact output
// order is not pinned by any fixture in the reference ("parity unpinned", see tests/test_contour.py).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <vector>

namespace py = pybind11;

namespace contour {

struct Pt { int x, y; };

// 8-neighbourhood, counter-clockwise on screen (row grows downward): E, NE, N, NW, W, SW, S, SE
static const int DI[8] = {0, -1, -1, -1, 0, 1, 1, 1};
static const int DJ[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static int dir_of(int di, int dj) {
  for (int k = 0; k < 8; ++k) if (DI[k] == di && DJ[k] == dj) return k;
  return -1;
}

struct Result {
  std::vector<std::vector<Pt>> contours;
  std::vector<std::array<int, 4>> hierarchy;   // next, prev, first_child, parent (OpenCV convention)
  std::vector<int> is_hole;
};

static std::vector<Pt> simplify_chain(const std::vector<Pt>& pts) {
  size_t n = pts.size();
  if (n <= 2) return pts;
  std::vector<Pt> out;
  for (size_t k = 0; k < n; ++k) {
    const Pt& a = pts[(k + n - 1) % n];
    const Pt& b = pts[k];
    const Pt& c = pts[(k + 1) % n];
    int d1x = b.x - a.x, d1y = b.y - a.y, d2x = c.x - b.x, d2y = c.y - b.y;
    if (d1x != d2x || d1y != d2y) out.push_back(b);
  }
  if (out.empty()) out.push_back(pts[0]);
  return out;
}

Result find_contours(const uint8_t* img, int H, int W, int thresh, bool simple) {
  const int Hp = H + 2, Wp = W + 2;
  std::vector<int32_t> f((size_t)Hp * Wp, 0);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) f[(size_t)(i + 1) * Wp + (j + 1)] = img[(size_t)i * W + j] > thresh ? 1 : 0;
  auto at = [&](int i, int j) -> int32_t& { return f[(size_t)i * Wp + j]; };

  Result R;
  std::vector<int> border_parent = {-1};   // index by NBD-1; NBD 1 = frame (a hole border)
  std::vector<int> border_hole = {1};
  std::vector<int> border_idx = {-1};      // contour index in R for NBD
  int nbd = 1;
  for (int i = 1; i < Hp - 1; ++i) {
    int lnbd = 1;
    for (int j = 1; j < Wp - 1; ++j) {
      int32_t fij = at(i, j);
      int i2 = 0, j2 = 0;
      bool start = false, hole = false;
      if (fij == 1 && at(i, j - 1) == 0) { start = true; hole = false; i2 = i; j2 = j - 1; }
      else if (fij >= 1 && at(i, j + 1) == 0) { start = true; hole = true; i2 = i; j2 = j + 1; if (fij > 1) lnbd = fij; }
      if (start) {
        ++nbd;
        // parent from LNBD (Suzuki table 1)
        int lb = lnbd - 1;
        int parent_nbd;
        if (!hole) parent_nbd = border_hole[lb] ? lnbd : (border_parent[lb] + 1);
        else parent_nbd = border_hole[lb] ? (border_parent[lb] + 1) : lnbd;
        border_parent.push_back(parent_nbd - 1);
        border_hole.push_back(hole ? 1 : 0);
        std::vector<Pt> pts;
        // 3.1 clockwise search from (i2,j2) around (i,j)
        int d0 = dir_of(i2 - i, j2 - j);
        int i1 = -1, j1 = -1;
        for (int k = 0; k < 8; ++k) {
          int d = (d0 - k + 8) % 8;
          if (at(i + DI[d], j + DJ[d]) != 0) { i1 = i + DI[d]; j1 = j + DJ[d]; break; }
        }
        if (i1 < 0) {
          at(i, j) = -nbd;
          pts.push_back({j - 1, i - 1});
        } else {
          i2 = i1; j2 = j1;
          int i3 = i, j3 = j;
          for (size_t guard = 0; guard < (size_t)Hp * Wp * 8; ++guard) {
            pts.push_back({j3 - 1, i3 - 1});
            int d = dir_of(i2 - i3, j2 - j3);
            int i4 = -1, j4 = -1;
            bool east_zero = false;
            for (int k = 1; k <= 8; ++k) {
              int dd = (d + k) % 8;
              int ni = i3 + DI[dd], nj = j3 + DJ[dd];
              if (at(ni, nj) != 0) { i4 = ni; j4 = nj; break; }
              if (dd == 0) east_zero = true;
            }
            if (east_zero) at(i3, j3) = -nbd;
            else if (at(i3, j3) == 1) at(i3, j3) = nbd;
            if (i4 == i && j4 == j && i3 == i1 && j3 == j1) break;
            i2 = i3; j2 = j3; i3 = i4; j3 = j4;
          }
        }
        border_idx.push_back((int)R.contours.size());
        R.contours.push_back(simple ? simplify_chain(pts) : pts);
        R.is_hole.push_back(hole ? 1 : 0);
        int pidx = border_parent.back() >= 0 ? border_idx[border_parent.back()] : -1;
        R.hierarchy.push_back({-1, -1, -1, pidx});
      }
      int32_t v = at(i, j);
      if (v != 1 && v != 0) lnbd = v < 0 ? -v : v;
    }
  }
  // sibling / child links
  std::vector<int> last_child(R.contours.size(), -1);
  int last_root = -1;
  for (int c = 0; c < (int)R.contours.size(); ++c) {
    int p = R.hierarchy[c][3];
    int& prev = p >= 0 ? last_child[p] : last_root;
    if (prev >= 0) { R.hierarchy[prev][0] = c; R.hierarchy[c][1] = prev; }
    else if (p >= 0) R.hierarchy[p][2] = c;
    prev = c;
  }
  return R;
}

double contour_area(const std::vector<Pt>& p, bool oriented = false) {
  double a = 0;
  size_t n = p.size();
  for (size_t k = 0; k < n; ++k) {
    const Pt& u = p[k];
    const Pt& v = p[(k + 1) % n];
    a += (double)u.x * v.y - (double)v.x * u.y;
  }
  a *= 0.5;
  return oriented ? a : std::fabs(a);
}

double arc_length(const std::vector<Pt>& p, bool closed) {
  double s = 0;
  size_t n = p.size();
  if (n < 2) return 0;
  for (size_t k = 0; k + 1 < n; ++k) s += std::hypot(p[k + 1].x - p[k].x, p[k + 1].y - p[k].y);
  if (closed) s += std::hypot(p[0].x - p[n - 1].x, p[0].y - p[n - 1].y);
  return s;
}

static void dp(const std::vector<Pt>& p, size_t a, size_t b, double eps, std::vector<char>& keep) {
  if (b <= a + 1) return;
  double dx = p[b].x - p[a].x, dy = p[b].y - p[a].y;
  double L = std::hypot(dx, dy);
  double best = -1; size_t bi = a;
  for (size_t k = a + 1; k < b; ++k) {
    double d = L > 0 ? std::fabs(dy * (p[k].x - p[a].x) - dx * (p[k].y - p[a].y)) / L
                     : std::hypot(p[k].x - p[a].x, p[k].y - p[a].y);
    if (d > best) { best = d; bi = k; }
  }
  if (best > eps) { keep[bi] = 1; dp(p, a, bi, eps, keep); dp(p, bi, b, eps, keep); }
}

std::vector<Pt> approx_poly(const std::vector<Pt>& p, double eps, bool closed) {
  size_t n = p.size();
  if (n < 3) return p;
  std::vector<Pt> q = p;
  size_t far = 0;
  if (closed) {   // split the closed curve at the point farthest from p[0]
    double best = -1;
    for (size_t k = 1; k < n; ++k) {
      double d = std::hypot(p[k].x - p[0].x, p[k].y - p[0].y);
      if (d > best) { best = d; far = k; }
    }
    q.push_back(p[0]);
  }
  std::vector<char> keep(q.size(), 0);
  keep[0] = 1; keep[q.size() - 1] = 1;
  if (closed) { keep[far] = 1; dp(q, 0, far, eps, keep); dp(q, far, q.size() - 1, eps, keep); }
  else dp(q, 0, q.size() - 1, eps, keep);
  std::vector<Pt> out;
  for (size_t k = 0; k < (closed ? q.size() - 1 : q.size()); ++k) if (keep[k]) out.push_back(q[k]);
  return out;
}

static std::vector<Pt> to_pts(py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
  auto r = a.unchecked<2>();
  std::vector<Pt> p;
  for (py::ssize_t k = 0; k < r.shape(0); ++k) p.push_back({r(k, 0), r(k, 1)});
  return p;
}

static py::array_t<int32_t> from_pts(const std::vector<Pt>& p) {
  py::array_t<int32_t> a({(py::ssize_t)p.size(), (py::ssize_t)2});
  auto w = a.mutable_unchecked<2>();
  for (size_t k = 0; k < p.size(); ++k) { w(k, 0) = p[k].x; w(k, 1) = p[k].y; }
  return a;
}

}  // namespace contour

void register_contour(py::module_& m) {
  auto c = m.def_submodule("contour", "Suzuki-Abe border following + contour geometry (cv2 subset)");
  c.def("find_contours", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img, int thresh, bool simple) {
    if (img.ndim() != 2) throw std::runtime_error("find_contours expects a 2-D uint8 image");
    auto R = contour::find_contours(img.data(), (int)img.shape(0), (int)img.shape(1), thresh, simple);
    py::list cs;
    for (auto& c : R.contours) cs.append(contour::from_pts(c));
    py::array_t<int32_t> h({(py::ssize_t)R.hierarchy.size(), (py::ssize_t)4});
    auto w = h.mutable_unchecked<2>();
    for (size_t k = 0; k < R.hierarchy.size(); ++k) for (int q = 0; q < 4; ++q) w(k, q) = R.hierarchy[k][q];
    return py::make_tuple(cs, h, R.is_hole);
  }, py::arg("img"), py::arg("thresh") = 127, py::arg("simple") = true);
  c.def("contour_area", [](py::array_t<int32_t> p, bool oriented) { return contour::contour_area(contour::to_pts(p), oriented); },
        py::arg("points"), py::arg("oriented") = false);
  c.def("arc_length", [](py::array_t<int32_t> p, bool closed) { return contour::arc_length(contour::to_pts(p), closed); },
        py::arg("points"), py::arg("closed") = true);
  c.def("approx_poly_dp", [](py::array_t<int32_t> p, double eps, bool closed) {
    return contour::from_pts(contour::approx_poly(contour::to_pts(p), eps, closed)); },
        py::arg("points"), py::arg("epsilon"), py::arg("closed") = true);
}
