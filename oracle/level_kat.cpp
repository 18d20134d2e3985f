// level_kat.cpp — known-answer generator for the level loader's transform and colour
// conversions, built against the reference's own header-only math library
// (deps/arklib/include/ark: quaternion.h rotateVector/quatToMatrix, transform.h
// translate/rotate/scale, color.h sRGB gammaDecode). Test infrastructure only: built
// by oracle/Makefile.ref into oracle/_ref/, its outputs are committed as
// tests/golden/level_kat.json by tests/golden/make_level_kat.py.
//
// stdin, one record per line:
//   T tx ty tz qx qy qz qw sx sy sz   -> forward right up (Transform.h:54-56) and the
//                                        local matrix translate * rotate * scale
//                                        (Transform.h:160-166), column-major
//   C r g b                            -> Color::fromNonLinearSRGB (color.h:426-430)
// Every number, in and out, is a float32 bit pattern as an 8-digit hex word (the
// loader's float32 values exactly, no decimal parsing on this side).
#include <cstdint>
#include <cstdio>
#include <cstring>

#include <ark/color.h>
#include <ark/quaternion.h>
#include <ark/transform.h>

static bool readWords(float* f, int n)
{
    for (int i = 0; i < n; ++i) {
        uint32_t u;
        if (std::scanf("%x", &u) != 1) return false;
        std::memcpy(&f[i], &u, 4);
    }
    return true;
}

static void word(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    std::printf(" %08x", u);
}

int main()
{
    char kind[4];
    while (std::scanf("%3s", kind) == 1) {
        if (kind[0] == 'T') {
            float t[3], q[4], s[3];
            if (!readWords(t, 3) || !readWords(q, 4) || !readWords(s, 3)) return 1;
            const ark::quat o(ark::vec3(q[0], q[1], q[2]), q[3]);
            const ark::vec3 fwd = ark::rotateVector(o, ark::globalForward);
            const ark::vec3 rgt = ark::rotateVector(o, ark::globalRight);
            const ark::vec3 up = ark::rotateVector(o, ark::globalUp);
            const ark::mat4 m = ark::translate(ark::vec3(t[0], t[1], t[2])) * ark::rotate(o) * ark::scale(ark::vec3(s[0], s[1], s[2]));
            std::printf("T");
            for (const ark::vec3& v : { fwd, rgt, up }) {
                word(v.x);
                word(v.y);
                word(v.z);
            }
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) word(m[c][r]);
            std::printf("\n");
        } else if (kind[0] == 'C') {
            float c[3];
            if (!readWords(c, 3)) return 1;
            const ark::Color col = ark::Color::fromNonLinearSRGB(ark::vec3(c[0], c[1], c[2]));
            std::printf("C");
            word(col.r());
            word(col.g());
            word(col.b());
            std::printf("\n");
        } else {
            return 1;
        }
    }
    return 0;
}
