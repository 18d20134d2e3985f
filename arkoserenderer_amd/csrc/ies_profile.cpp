// IES photometric profiles -> spot-light LUTs (include/ark_ies.h).
//
// Host-side C++: the LUT is built once per light when the scene is assembled
// (GpuScene.cpp:1101-1124) and uploaded as an R32F texture, so there is nothing to
// accelerate here; what matters is that the table is the reference's, value for
// value. Parsing follows IESProfile::parse (IESProfile.cpp:57-175) on top of
// ParseContext (arkcore/utility/ParseContext.cpp: getline for lines, operator>> for
// numbers, optional ',' between array values); lookups follow lookupValue /
// computeLookupLocation / getValue (:177-333) in fp32, lerp(a, b, t) = (1-t)a + tb
// (ark/core.h:140-143).
#include "../../include/ark_ies.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <vector>

namespace {

thread_local std::string g_lastError;

struct IesProfile {
    ArkIesInfo info {};
    std::vector<float> anglesV, anglesH, candela; // candela[v + nV * h]
};

// ParseContext::consumeDelimiter(',', true)
void skipDelimiter(std::istream& in)
{
    while (std::isspace(in.peek())) in.get();
    if (in.peek() == ',') in.get();
    while (std::isspace(in.peek())) in.get();
}

bool fail(const char* what)
{
    g_lastError = what;
    return false;
}

bool parseProfile(const std::string& text, IesProfile& p)
{
    std::istringstream in(text);
    std::string line;
    std::getline(in, line);
    if (line != "IESNA91" && line != "IESNA:LM-63-1995" && line != "IESNA:LM-63-2002") return fail("invalid version line");
    std::string tilt;
    std::getline(in, tilt);
    while (!tilt.empty() && tilt[0] == '[') { // keyword lines
        if (!std::getline(in, tilt)) return fail("no TILT line");
    }
    if (tilt.rfind("TILT=NONE", 0) != 0) return fail("only TILT=NONE is supported");

    auto readInt = [&](int& v) { return static_cast<bool>(in >> v); };
    auto readFloat = [&](float& v) { return static_cast<bool>(in >> v); };
    ArkIesInfo& I = p.info;
    float multiplier = 0.0f, futureUse = 0.0f;
    int nV = 0, nH = 0;
    if (!readInt(I.lamp_count) || !readFloat(I.lumens_per_lamp) || !readFloat(multiplier) || !readInt(nV) || !readInt(nH) ||
        !readInt(I.photometric_type) || !readInt(I.units_type) || !readFloat(I.width) || !readFloat(I.length) || !readFloat(I.height) ||
        !readFloat(I.ballast_factor) || !readFloat(futureUse) || !readFloat(I.input_watts))
        return fail("truncated header");
    if (I.lamp_count <= 0) return fail("invalid lamp count");
    if (!(multiplier > 0.0f)) return fail("candela multiplier must be greater than zero");
    if (nV < 1 || nH < 1) return fail("number of vertical and horizontal angles must be greater than zero");
    if (I.photometric_type < 1 || I.photometric_type > 3) return fail("invalid photometric type");
    if (I.units_type != 1 && I.units_type != 2) return fail("bad units type");
    I.num_angles_v = static_cast<uint32_t>(nV);
    I.num_angles_h = static_cast<uint32_t>(nH);

    auto readAngles = [&](int n, float hi, std::vector<float>& out) {
        float last = -std::numeric_limits<float>::infinity();
        for (int i = 0; i < n; ++i) {
            float a;
            if (!readFloat(a)) return fail("truncated angle list");
            if (!(a >= 0.0f && a <= hi)) return fail("angle out of range");
            if (a <= last) return fail("angles must be strictly increasing");
            out.push_back(a);
            last = a;
            skipDelimiter(in);
        }
        return true;
    };
    if (!readAngles(nV, 180.0f, p.anglesV) || !readAngles(nH, 360.0f, p.anglesH)) return false;
    const size_t count = static_cast<size_t>(nV) * static_cast<size_t>(nH);
    p.candela.reserve(count);
    I.max_candela = 0.0f;
    for (size_t i = 0; i < count; ++i) {
        float v;
        if (!readFloat(v)) return fail("truncated candela values");
        p.candela.push_back(multiplier * v);
        I.max_candela = std::fmax(I.max_candela, p.candela.back());
        skipDelimiter(in);
    }
    I.first_angle_v = p.anglesV.front();
    I.last_angle_v = p.anglesV.back();
    I.first_angle_h = p.anglesH.front();
    I.last_angle_h = p.anglesH.back();
    return true;
}

// Fractional index of `angle` in the increasing list (computeLookupLocation).
float fractionalIndex(float angle, const std::vector<float>& list)
{
    int lo = 0, hi = static_cast<int>(list.size()) - 1;
    if (angle <= list[lo]) return 0.0f;
    if (angle >= list[hi]) return static_cast<float>(hi);
    while (lo < hi) {
        if (hi - lo == 1) {
            const float span = list[hi] - list[lo];
            if (span < 1e-3f) return static_cast<float>(lo);
            return static_cast<float>(lo) + (angle - list[lo]) / span;
        }
        const int mid = (lo + hi + 1) / 2;
        const float m = list[mid];
        if (angle == m) return static_cast<float>(mid);
        if (angle > m) lo = mid;
        else hi = mid;
    }
    return static_cast<float>(lo);
}

float lerpf(float a, float b, float t) { return (1.0f - t) * a + t * b; }

// getValue: bilinear over (horizontal, vertical) index space, indices clamped.
float sampleCandela(const IesProfile& p, float locH, float locV)
{
    const int nH = static_cast<int>(p.anglesH.size()), nV = static_cast<int>(p.anglesV.size());
    auto at = [&](int h, int v) {
        h = std::max(0, std::min(h, nH - 1));
        v = std::max(0, std::min(v, nV - 1));
        return p.candela[static_cast<size_t>(v) + static_cast<size_t>(nV) * static_cast<size_t>(h)];
    };
    const int h = static_cast<int>(locH), v = static_cast<int>(locV);
    const float dh = locH - static_cast<float>(h), dv = locV - static_cast<float>(v);
    const float lower = lerpf(at(h, v), at(h + 1, v), dh);
    const float upper = lerpf(at(h, v + 1), at(h + 1, v + 1), dh);
    return lerpf(lower, upper, dv);
}

// lookupValue: the photometric type's symmetry folds the horizontal angle.
bool lookup(const IesProfile& p, float angleH, float angleV, float* out)
{
    float h = angleH;
    switch (p.info.photometric_type) {
    case 3: break; // Type A
    case 2: return fail("Type B IES profiles are not implemented");
    case 1: {
        const long last = std::lround(p.anglesH.back());
        if (p.anglesH.size() == 1 && last == 0) {
            h = 0.0f; // laterally symmetric
        } else if (last == 90) {
            h = std::fmod(angleH, 90.0f); // symmetric per quadrant
            const int quadrant = static_cast<int>(angleH / 90.0f);
            if (quadrant == 1 || quadrant == 3) h = 90.0f - h;
        } else if (last == 180) {
            h = std::fmod(angleH, 180.0f); // bilateral about the 0-180 plane
            if (angleH >= 180.0f) h = 360.0f - angleH;
        } else if (last > 180 && last <= 360) {
            h = angleH; // no lateral symmetry
        } else {
            return fail("invalid last horizontal angle");
        }
        break;
    }
    default: return fail("invalid photometric type");
    }
    *out = sampleCandela(p, fractionalIndex(h, p.anglesH), fractionalIndex(angleV, p.anglesV));
    return true;
}

int buildLut(const std::string& text, uint32_t size, float* lut, ArkIesInfo* info)
{
    g_lastError.clear();
    if (!lut || size == 0) return ARK_IES_E_INVALID_ARGUMENT;
    IesProfile p;
    if (!parseProfile(text, p)) return ARK_IES_E_PARSE;
    // assembleLookupTextureData: row y = horizontal, column x = vertical
    for (uint32_t y = 0; y < size; ++y) {
        const float horizontal = static_cast<float>(y) / static_cast<float>(size) * 360.0f;
        for (uint32_t x = 0; x < size; ++x) {
            const float vertical = static_cast<float>(x) / static_cast<float>(size) * 180.0f;
            if (!lookup(p, horizontal, vertical, &lut[static_cast<size_t>(y) * size + x])) return ARK_IES_E_PARSE;
        }
    }
    if (info) *info = p.info;
    return ARK_IES_OK;
}

} // namespace

extern "C" {

int ark_ies_lut_from_memory(const char* text, uint64_t length, uint32_t lut_size, float* out_lut, ArkIesInfo* out_info)
{
    if (!text) return ARK_IES_E_INVALID_ARGUMENT;
    return buildLut(std::string(text, static_cast<size_t>(length)), lut_size, out_lut, out_info);
}

int ark_ies_lut_from_file(const char* path, uint32_t lut_size, float* out_lut, ArkIesInfo* out_info)
{
    if (!path) return ARK_IES_E_INVALID_ARGUMENT;
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) {
        g_lastError = std::string("could not read ") + path;
        return ARK_IES_E_IO;
    }
    std::ostringstream ss;
    ss << f.rdbuf();
    return buildLut(ss.str(), lut_size, out_lut, out_info);
}

int ark_ies_lookup(const char* text, uint64_t length, float angle_h, float angle_v, float* out_value)
{
    g_lastError.clear();
    if (!text || !out_value) return ARK_IES_E_INVALID_ARGUMENT;
    IesProfile p;
    if (!parseProfile(std::string(text, static_cast<size_t>(length)), p)) return ARK_IES_E_PARSE;
    return lookup(p, angle_h, angle_v, out_value) ? ARK_IES_OK : ARK_IES_E_PARSE;
}

const char* ark_ies_last_error(void) { return g_lastError.c_str(); }

} // extern "C"
