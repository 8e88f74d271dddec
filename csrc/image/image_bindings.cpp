// pybind11 module _image: host image stages on numpy HWC uint8 arrays and the
// device entry points on raw pointers (torch tensors' data_ptr + stream).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>

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

}  // namespace

PYBIND11_MODULE(_image, m) {
  m.doc() = "MI355X image kernels (resize/crop/color/normalize fused preprocess, blur, threshold, gaussian, flip)";
  m.def("gpu_available", &ImageGpuAvailable);
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
