// ref_bench.cpp — timing harness for the reference C++ decoder (TEST / BASELINE INFRASTRUCTURE).
//
// Built by oracle/Makefile against the reference's own sources under /root/reference/cpp-decoder
// (never copied into this repo).  Times JPEGParser::extract() + decode() exactly as the reference's
// Google-Benchmark harness does (cpp-decoder/benchmark/benchmark.cc:29-35): the constructor (file
// read) and write() (.array text dump) stay outside the timed region.
//
// usage: ref_bench <reps> <file.jpg>...   -> one JSON line {"images":N,"reps":R,"seconds":S,...}
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "src/parser.h"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <reps> <file.jpg>...\n", argv[0]);
        return 2;
    }
    int reps = std::atoi(argv[1]);
    double total = 0.0;
    long long pixels = 0;
    int images = 0;
    for (int r = 0; r < reps; r++) {
        for (int i = 2; i < argc; i++) {
            std::string path = argv[i];
            JPEGParser parser(path);
            auto t0 = std::chrono::high_resolution_clock::now();
            parser.extract();
            parser.decode();
            auto t1 = std::chrono::high_resolution_clock::now();
            total += std::chrono::duration<double>(t1 - t0).count();
            images++;
        }
    }
    (void)pixels;
    std::printf("{\"images\": %d, \"reps\": %d, \"seconds\": %.6f}\n", images, reps, total);
    return 0;
}
