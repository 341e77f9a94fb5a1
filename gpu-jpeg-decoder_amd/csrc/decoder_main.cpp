// decoder_main.cpp — CLI `decoder [--fancy] [--ppm] <jpeg> [outdir]`, mirroring the reference CLIs
// (cpp-decoder/main.cpp:5-16 and cuda-decoder/main.cu:7-40): extract, decode, write `.array`.
// --fancy selects triangular chroma upsampling (JD_FLAG_FANCY_UPSAMPLING); --ppm writes the binary
// PPM of the reference's libjpeg comparison flow (testing/jpeglib_output_ppm/) instead.
#include <cstdio>
#include <exception>
#include <string>

#include "jpeg_parser.hpp"

int main(int argc, char* argv[]) {
    bool ppm = false;
    while (argc >= 2 && argv[1][0] == '-' && argv[1][1] == '-') {
        const std::string opt = argv[1];
        if (opt == "--fancy") jdamd::default_context_flags() |= JD_FLAG_FANCY_UPSAMPLING;
        else if (opt == "--ppm") ppm = true;
        else {
            std::fprintf(stderr, "decoder: unknown option %s\n", opt.c_str());
            return 1;
        }
        argv++;
        argc--;
    }
    if (argc < 2) {
        std::printf("Please provide the name of the image file to be decompressed.\n");
        return 1;
    }
    try {
        jdamd::JPEGParser parser(argv[1]);
        parser.extract();
        parser.decode();
        if (ppm) parser.write_ppm(argc >= 3 ? argv[2] : ".");
        else if (argc >= 3) parser.write(argv[2]);
        else parser.write();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "decoder: %s\n", e.what());
        return 1;
    }
    return 0;
}
