// jpeg_parser.hpp — C++ mirror of the reference's CPU-side interface, built on the C ABI.
//
// Reference: class JPEGParser { JPEGParser(path); extract(); decode(); write(); }
// (cpp-decoder/src/parser.h:42-69, used by cpp-decoder/main.cpp:5-16 and by the Google-Benchmark
// harness cpp-decoder/benchmark/benchmark.cc:31-36).  Same call sequence and meaning; decode() runs
// on the GPU through libjdamd.so.  Errors throw std::runtime_error, as the reference's CUDA host
// code does for runtime failures (cuda-decoder/src/parser.cu:317-321).
#pragma once

#include <fstream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <vector>

#include "jd.h"

namespace jdamd {

// Context flags for the process-wide context (set before the first decode), e.g.
// JD_FLAG_FANCY_UPSAMPLING for the CLI's --fancy.
inline unsigned& default_context_flags() {
    static unsigned flags = 0;
    return flags;
}

inline jd_ctx* default_context() {
    static jd_ctx* ctx = [] {
        jd_ctx* c = nullptr;
        jd_opts o{default_context_flags(), 0};
        jd_status st = jd_ctx_create(&c, 0, &o);
        if (st != JD_OK) throw std::runtime_error(std::string("jd_ctx_create: ") + jd_status_str(st));
        return c;
    }();
    return ctx;
}

class JPEGParser {
  public:
    explicit JPEGParser(const std::string& imagePath) : path_(imagePath) {
        std::ifstream in(imagePath, std::ios::binary);
        if (!in) throw std::runtime_error("cannot open " + imagePath);
        bytes_.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
        const size_t slash = imagePath.find_last_of('/');
        filename_ = slash == std::string::npos ? imagePath : imagePath.substr(slash + 1);
    }

    // parser.cpp:24-103: marker walk -> dimensions, tables, ECS location.
    void extract() {
        jd_status st = jd_parse(bytes_.data(), bytes_.size(), &hdr_);
        if (st != JD_OK) throw std::runtime_error(filename_ + ": " + jd_status_str(st));
        extracted_ = true;
    }

    // parser.cpp:144-195: entropy decode, IDCT, colour conversion (on the GPU).
    void decode() {
        if (!extracted_) extract();
        rgb_.assign(size_t(hdr_.width) * hdr_.height * 3, 0);
        int w = 0, h = 0;
        jd_status st = jd_decode(default_context(), bytes_.data(), bytes_.size(), rgb_.data(), 0, &w, &h);
        if (st != JD_OK) throw std::runtime_error(filename_ + ": " + jd_status_str(st));
    }

    // parser.cpp:197-209: "<outdir>/<name>.array" (the reference hard-codes
    // ../testing/cpp_output_arrays; testing/compare.py:41-43 expects "<impl>_output_arrays").
    void write(const std::string& outdir = "../testing/gpu_output_arrays") const {
        const std::string out = outdir + "/" + stem() + ".array";
        jd_status st = jd_write_array(out.c_str(), rgb_.data(), hdr_.width, hdr_.height);
        if (st != JD_OK) throw std::runtime_error(out + ": " + jd_status_str(st));
    }

    // The libjpeg comparison format of the reference's testing flow (testing/jpeglib_output_ppm/,
    // jpeglib-implementation/process_ppm.py): "<outdir>/<name>.ppm", binary P6.
    void write_ppm(const std::string& outdir) const {
        const std::string out = outdir + "/" + stem() + ".ppm";
        jd_status st = jd_write_ppm(out.c_str(), rgb_.data(), hdr_.width, hdr_.height);
        if (st != JD_OK) throw std::runtime_error(out + ": " + jd_status_str(st));
    }

    int width() const { return hdr_.width; }
    int height() const { return hdr_.height; }
    const std::vector<uint8_t>& rgb() const { return rgb_; }
    const jd_header& header() const { return hdr_; }

  private:
    std::string stem() const {
        const size_t dot = filename_.find_last_of('.');
        return dot == std::string::npos ? filename_ : filename_.substr(0, dot);
    }
    std::string path_, filename_;
    std::vector<uint8_t> bytes_;
    std::vector<uint8_t> rgb_;
    jd_header hdr_{};
    bool extracted_ = false;
};

}  // namespace jdamd
