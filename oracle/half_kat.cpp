// half_kat.cpp — known-answer generator for fp32 -> fp16 conversion using the
// reference's own in-tree fp16 library (deps/half/half.hpp, round_to_nearest).
// Reads raw float32 from stdin, writes raw uint16 half bits to stdout.
// Built by oracle/Makefile.ref into oracle/_ref/ (never shipped, test-only).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include <half.hpp>

int main()
{
    std::vector<float> in;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, sizeof(float), 4096, stdin)) > 0) in.insert(in.end(), buf, buf + n);
    std::vector<uint16_t> out(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        half_float::half h(in[i]);
        std::memcpy(&out[i], &h, 2);
    }
    std::fwrite(out.data(), 2, out.size(), stdout);
    return 0;
}
