// decoder_main.cpp — CLI `decoder [--fancy] <jpeg> [outdir]`, mirroring the reference CLIs
// (cpp-decoder/main.cpp:5-16 and cuda-decoder/main.cu:7-40): extract, decode, write `.array`.
// --fancy selects triangular chroma upsampling (JD_FLAG_FANCY_UPSAMPLING).
#include <cstdio>
#include <exception>
#include <string>

#include "jpeg_parser.hpp"

int main(int argc, char* argv[]) {
    if (argc >= 2 && std::string(argv[1]) == "--fancy") {
        jdamd::default_context_flags() |= JD_FLAG_FANCY_UPSAMPLING;
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
        if (argc >= 3) parser.write(argv[2]);
        else parser.write();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "decoder: %s\n", e.what());
        return 1;
    }
    return 0;
}
