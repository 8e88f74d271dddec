// pybind11 module _image: host image stages on numpy HWC uint8 arrays and the
// device entry points on raw pointers (torch tensors' data_ptr + stream).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "image_cpu.h"
#include "jpeg_decode.h"

namespace py = pybind11;
using namespace smlimg;
using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

namespace {

struct HWC {
  int h, w, c;
};

HWC Dims(const U8& a) {
  if (a.ndim() == 2) return {static_cast<int>(a.shape(0)), static_cast<int>(a.shape(1)), 1};
  if (a.ndim() == 3) return {static_cast<int>(a.shape(0)), static_cast<int>(a.shape(1)), static_cast<int>(a.shape(2))};
  throw std::invalid_argument("expected an HxW or HxWxC uint8 image");
}

U8 NewImage(int h, int w, int c) {
  if (c == 1) return U8({h, w});
  return U8({h, w, c});
}

template <class T>
T* Ptr(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

// A fixed team of helper threads for the host copies around a device batch (image rows into a pinned slot,
// results out into per-row objects): one Python task per image cost more than its 150-786 KB copy (r6 pass 19:
// 2048 futures ~50 ms of a 134 ms transform), and numpy's tobytes holds the GIL for its memcpy.
class Team {
 public:
  static Team& Get() {
    static Team* t = new Team();  // never destroyed (teardown order)
    return *t;
  }
  int size() const { return static_cast<int>(th_.size()) + 1; }
  // fn(t) for t in [0, size()), t = 0 on the calling thread (no GIL needed by fn)
  void Run(const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> run(run_mu_);  // one job at a time
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      pending_ = static_cast<int>(th_.size());
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  Team() {
    const unsigned hw = std::thread::hardware_concurrency();
    const int n = std::max(1, std::min(16, hw ? static_cast<int>(hw) : 1));
    for (int t = 1; t < n; ++t) th_.emplace_back([this, t] { Loop(t); });
  }
  void Loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        job = job_;
      }
      (*job)(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(int)>* job_ = nullptr;
  int pending_ = 0;
  uint64_t gen_ = 0;
};

// copies (dst[i] <- src[i], len[i] bytes) spread over the team by bytes, the GIL released
void CopyMany(const std::vector<char*>& dst, const std::vector<const char*>& src, const std::vector<size_t>& len) {
  const size_t n = dst.size();
  if (n == 0) return;
  size_t total = 0;
  for (size_t l : len) total += l;
  Team& team = Team::Get();
  const int nt = team.size();
  if (nt == 1 || total < (size_t(1) << 20)) {
    for (size_t i = 0; i < n; ++i) std::memcpy(dst[i], src[i], len[i]);
    return;
  }
  // thread t copies the byte range [total * t / nt, total * (t + 1) / nt) of the concatenated copies
  std::vector<size_t> start(n + 1, 0);
  for (size_t i = 0; i < n; ++i) start[i + 1] = start[i] + len[i];
  py::gil_scoped_release rel;
  team.Run([&](int t) {
    const size_t a = total * t / nt, b = total * (t + 1) / nt;
    size_t i = std::upper_bound(start.begin(), start.end(), a) - start.begin() - 1;
    for (size_t p = a; p < b && i < n; ++i) {
      const size_t e = std::min(b, start[i + 1]);
      std::memcpy(dst[i] + (p - start[i]), src[i] + (p - start[i]), e - p);
      p = e;
    }
  });
}

}  // namespace

PYBIND11_MODULE(_image, m) {
  m.doc() = "MI355X image kernels (resize/crop/color/normalize fused preprocess, blur, threshold, gaussian, flip)";
  m.def("gpu_available", &ImageGpuAvailable);
  // host side of a device batch: n images (bytes / contiguous uint8 arrays) into one buffer, image i at
  // i * item_bytes (every image that size), or back to back when item_bytes == 0
  m.def("gather_into", [](const std::vector<py::buffer>& srcs, uintptr_t dst, size_t item_bytes) {
    std::vector<char*> d;
    std::vector<const char*> s;
    std::vector<size_t> l;
    std::vector<py::buffer_info> keep;  // buffer views held until the copies are done
    keep.reserve(srcs.size());
    size_t packed = 0;
    for (size_t i = 0; i < srcs.size(); ++i) {
      keep.push_back(srcs[i].request());
      const py::buffer_info& bi = keep.back();
      const size_t nb = static_cast<size_t>(bi.size) * static_cast<size_t>(bi.itemsize);
      if (item_bytes && nb != item_bytes)
        throw std::invalid_argument("gather_into: an image has " + std::to_string(nb) + " bytes, expected " +
                                    std::to_string(item_bytes));
      bool contiguous = true;
      for (ssize_t k = bi.ndim - 1, want = bi.itemsize; k >= 0; --k) {
        if (bi.shape[k] > 1 && bi.strides[k] != want) contiguous = false;
        want *= bi.shape[k];
      }
      if (!contiguous) throw std::invalid_argument("gather_into: a non-contiguous image");
      d.push_back(reinterpret_cast<char*>(dst) + (item_bytes ? i * item_bytes : packed));
      packed += nb;
      s.push_back(static_cast<const char*>(bi.ptr));
      l.push_back(nb);
    }
    CopyMany(d, s, l);
  });
  // result side: n per-row bytes objects (item_bytes each) filled from one buffer in parallel
  m.def("split_bytes", [](uintptr_t src, size_t n, size_t item_bytes) {
    py::list out(n);
    std::vector<char*> d(n);
    std::vector<const char*> s(n);
    std::vector<size_t> l(n, item_bytes);
    for (size_t i = 0; i < n; ++i) {
      PyObject* b = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(item_bytes));
      if (!b) throw py::error_already_set();
      d[i] = PyBytes_AS_STRING(b);
      s[i] = reinterpret_cast<const char*>(src) + i * item_bytes;
      PyList_SET_ITEM(out.ptr(), static_cast<Py_ssize_t>(i), b);  // steals the reference
    }
    CopyMany(d, s, l);  // the objects are not visible to other threads until this returns
    return out;
  });
  // one buffer into another (the float-tensor results out of a reused pinned slot)
  m.def("copy_parallel", [](uintptr_t dst, uintptr_t src, size_t bytes) {
    CopyMany({reinterpret_cast<char*>(dst)}, {reinterpret_cast<const char*>(src)}, {bytes});
  });
  m.def("resize", [](U8 img, int h, int w) {
    HWC d = Dims(img);
    U8 out = NewImage(h, w, d.c);
    {
      py::gil_scoped_release rel;
      ResizeHost(img.data(), d.h, d.w, d.c, out.mutable_data(), h, w);
    }
    return out;
  });
  m.def("box_blur", [](U8 img, int kw, int kh) {
    HWC d = Dims(img);
    U8 out = NewImage(d.h, d.w, d.c);
    {
      py::gil_scoped_release rel;
      BoxBlurHost(img.data(), d.h, d.w, d.c, out.mutable_data(), kw, kh);
    }
    return out;
  });
  m.def("gaussian_kernel", &GaussianKernel);
  m.def("column_filter", [](U8 img, std::vector<double> k) {
    HWC d = Dims(img);
    U8 out = NewImage(d.h, d.w, d.c);
    {
      py::gil_scoped_release rel;
      ColumnFilterHost(img.data(), d.h, d.w, d.c, out.mutable_data(), k.data(), static_cast<int>(k.size()));
    }
    return out;
  });
  m.def("threshold", [](U8 img, double thr, double maxval, int type) {
    HWC d = Dims(img);
    U8 out = NewImage(d.h, d.w, d.c);
    ThresholdHost(img.data(), static_cast<int64_t>(d.h) * d.w * d.c, out.mutable_data(), thr, maxval, type);
    return out;
  });
  m.def("cvt_color", [](U8 img, int code) {
    HWC d = Dims(img);
    const int co = CvtChannelsOut(code, d.c);
    U8 out = NewImage(d.h, d.w, co);
    CvtColorHost(img.data(), static_cast<int64_t>(d.h) * d.w, d.c, code, out.mutable_data());
    return out;
  });
  m.def("cvt_channels_out", &CvtChannelsOut);
  m.def("to_tensor", [](U8 img, std::vector<int> chan_map, double scale, std::vector<double> mean,
                        std::vector<double> stdv) {
    HWC d = Dims(img);
    const int co = static_cast<int>(chan_map.size());
    if (static_cast<int>(mean.size()) != co || static_cast<int>(stdv.size()) != co)
      throw std::invalid_argument("mean/std length must equal the number of output channels");
    py::array_t<float> out({co, d.h, d.w});
    ToTensorHost(img.data(), d.h, d.w, d.c, chan_map.data(), co, scale, mean.data(), stdv.data(), out.mutable_data());
    return out;
  });

  // ---------------------------------------------------------------- JPEG decode
  m.def("jpeg_probe", [](const std::vector<py::bytes>& files) {
    const py::ssize_t n = static_cast<py::ssize_t>(files.size());
    py::array_t<int32_t> out({n, py::ssize_t(4)});  // height, width, channels, supported
    auto o = out.mutable_unchecked<2>();
    for (py::ssize_t i = 0; i < n; ++i) {
      char* p = nullptr;
      py::ssize_t len = 0;
      PyBytes_AsStringAndSize(files[i].ptr(), &p, &len);
      JpegInfo info = JpegProbe(reinterpret_cast<const uint8_t*>(p), static_cast<size_t>(len));
      o(i, 0) = info.height; o(i, 1) = info.width; o(i, 2) = info.channels; o(i, 3) = info.supported ? 1 : 0;
    }
    return out;
  });
  m.def("jpeg_decode", [](py::bytes data) -> py::object {
    char* p = nullptr;
    py::ssize_t len = 0;
    PyBytes_AsStringAndSize(data.ptr(), &p, &len);
    JpegInfo info = JpegProbe(reinterpret_cast<const uint8_t*>(p), static_cast<size_t>(len));
    if (!info.supported) return py::none();
    U8 out = NewImage(info.height, info.width, info.channels);
    std::string why;
    uint8_t* dst = out.mutable_data();
    const size_t cap = static_cast<size_t>(out.nbytes());
    bool ok;
    {
      py::gil_scoped_release rel;
      ok = JpegDecode(reinterpret_cast<const uint8_t*>(p), static_cast<size_t>(len), dst, cap, &why);
    }
    if (!ok) return py::none();
    return std::move(out);
  });
  // batch decode straight into a caller-owned buffer (e.g. pinned host memory): image i -> out + offsets[i],
  // sizes[i] bytes reserved (from jpeg_probe); returns per-image success flags (0 -> caller falls back)
  m.def("jpeg_decode_into", [](const std::vector<py::bytes>& files, uintptr_t out, uint64_t out_len,
                               std::vector<int64_t> offsets, std::vector<int64_t> sizes, int threads) {
    const size_t n = files.size();
    if (offsets.size() != n || sizes.size() != n) throw std::invalid_argument("offsets / sizes length mismatch");
    std::vector<const uint8_t*> ptrs(n);
    std::vector<size_t> lens(n);
    for (size_t i = 0; i < n; ++i) {
      char* p = nullptr;
      py::ssize_t len = 0;
      PyBytes_AsStringAndSize(files[i].ptr(), &p, &len);
      ptrs[i] = reinterpret_cast<const uint8_t*>(p);
      lens[i] = static_cast<size_t>(len);
      if (offsets[i] >= 0 && (sizes[i] < 0 || static_cast<uint64_t>(offsets[i]) + static_cast<uint64_t>(sizes[i]) > out_len))
        throw std::invalid_argument("jpeg_decode_into: image slot outside the output buffer");
    }
    py::array_t<uint8_t> ok(static_cast<py::ssize_t>(n));
    uint8_t* okp = ok.mutable_data();
    {
      py::gil_scoped_release rel;
      JpegDecodeBatch(ptrs, lens, Ptr<uint8_t>(out), offsets, sizes, okp, threads);
    }
    return ok;
  });

  // ---------------------------------------------------------------- device
  m.def("preprocess_batch_device",
        [](uintptr_t src, uintptr_t offsets, uintptr_t dims, int B, int out_h, int out_w, int resize_h, int resize_w,
           int crop_y, int crop_x, std::vector<int> chan_map, double scale, std::vector<double> mean,
           std::vector<double> stdv, int out_dtype, int nhwc, uintptr_t out, uintptr_t stream,
           std::vector<int32_t> host_dims) {
          PrepParams p{};
          if (resize_h > 0 && host_dims.size() != static_cast<size_t>(3) * B)
            throw std::invalid_argument("preprocess: resize needs host_dims = 3 ints per image");
          p.out_h = out_h; p.out_w = out_w; p.resize_h = resize_h; p.resize_w = resize_w;
          p.crop_y = crop_y; p.crop_x = crop_x;
          p.cout = static_cast<int>(chan_map.size());
          if (p.cout < 1 || p.cout > 4 || mean.size() != chan_map.size() || stdv.size() != chan_map.size())
            throw std::invalid_argument("preprocess: bad channel map / mean / std");
          for (int k = 0; k < p.cout; ++k) { p.chan_map[k] = chan_map[k]; p.mean[k] = mean[k]; p.stdv[k] = stdv[k]; }
          p.scale = scale; p.out_dtype = out_dtype; p.nhwc = nhwc;
          p.host_dims = host_dims.empty() ? nullptr : host_dims.data();
          PreprocessBatchDevice(Ptr<const uint8_t>(src), Ptr<const int64_t>(offsets), Ptr<const int32_t>(dims), B, p,
                                Ptr<void>(out), Ptr<void>(stream));
        }, py::arg("src"), py::arg("offsets"), py::arg("dims"), py::arg("B"), py::arg("out_h"), py::arg("out_w"),
        py::arg("resize_h"), py::arg("resize_w"), py::arg("crop_y"), py::arg("crop_x"), py::arg("chan_map"),
        py::arg("scale"), py::arg("mean"), py::arg("stdv"), py::arg("out_dtype"), py::arg("nhwc"), py::arg("out"),
        py::arg("stream"), py::arg("host_dims") = std::vector<int32_t>{});
  m.def("crop_flip_batch_device", [](uintptr_t src, int B, int sh, int sw, int c, uintptr_t dst, int dh, int dw, int cy,
                                     int cx, int flip, uintptr_t stream) {
    CropFlipBatchDevice(Ptr<const uint8_t>(src), B, sh, sw, c, Ptr<uint8_t>(dst), dh, dw, cy, cx, flip, Ptr<void>(stream));
  });
  m.def("resize_batch_device", [](uintptr_t src, int B, int sh, int sw, int c, uintptr_t dst, int dh, int dw,
                                  uintptr_t stream) {
    ResizeBatchDevice(Ptr<const uint8_t>(src), B, sh, sw, c, Ptr<uint8_t>(dst), dh, dw, Ptr<void>(stream));
  });
  m.def("box_blur_batch_device", [](uintptr_t src, int B, int h, int w, int c, uintptr_t dst, int kw, int kh,
                                    uintptr_t stream) {
    BoxBlurBatchDevice(Ptr<const uint8_t>(src), B, h, w, c, Ptr<uint8_t>(dst), kw, kh, Ptr<void>(stream));
  });
  m.def("column_filter_batch_device", [](uintptr_t src, int B, int h, int w, int c, uintptr_t dst,
                                         std::vector<double> k, uintptr_t stream) {
    ColumnFilterBatchDevice(Ptr<const uint8_t>(src), B, h, w, c, Ptr<uint8_t>(dst), k.data(),
                            static_cast<int>(k.size()), Ptr<void>(stream));
  });
  m.def("threshold_device", [](uintptr_t src, int64_t n, uintptr_t dst, double thr, double maxval, int type,
                               uintptr_t stream) {
    ThresholdDevice(Ptr<const uint8_t>(src), n, Ptr<uint8_t>(dst), thr, maxval, type, Ptr<void>(stream));
  });
  m.def("flip_batch_device", [](uintptr_t src, int B, int h, int w, int c, uintptr_t dst, int code, uintptr_t stream) {
    FlipBatchDevice(Ptr<const uint8_t>(src), B, h, w, c, Ptr<uint8_t>(dst), code, Ptr<void>(stream));
  });
  m.def("cvt_color_device", [](uintptr_t src, int64_t npx, int cin, int code, uintptr_t dst, uintptr_t stream) {
    CvtColorDevice(Ptr<const uint8_t>(src), npx, cin, code, Ptr<uint8_t>(dst), Ptr<void>(stream));
  });
}
