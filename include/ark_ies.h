/* ark_ies.h - IES photometric profile -> spot-light lookup table (C-ABI).
 *
 * Replaces IESProfile (arkcore/asset/external/IESProfile.{h,cpp}: parse :57-175,
 * lookupValue :177-257, computeLookupLocation :259-306, getValue :308-333,
 * assembleLookupTextureData :335-352) and the LUT upload of
 * GpuScene::registerLight (arkose/rendering/GpuScene.cpp:1101-1124: 256 x 256 R32F,
 * linear filter, clamp to edge). The LUT feeds ArkSpotLight.ies_profile_index as an
 * ARK_TEX_R32F texture with ARK_WRAP_CLAMP_TO_EDGE; the shading kernels sample it as
 * evaluateIESLookupTable (lighting.glsl:20-39) does.
 *
 * Where the reference logs Fatal (bad version, TILT other than NONE, non-positive
 * lamp count or candela multiplier, bad photometric/units type, angles not strictly
 * increasing, Type B profiles, an unsupported last horizontal angle) these return
 * ARK_IES_E_PARSE and leave the reason in ark_ies_last_error(). */
#ifndef ARK_IES_H
#define ARK_IES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARK_IES_OK 0
#define ARK_IES_E_INVALID_ARGUMENT (-1)
#define ARK_IES_E_IO (-2)
#define ARK_IES_E_PARSE (-3)

#define ARK_IES_LUT_SIZE 256 /* GpuScene.cpp:1104 */

typedef struct ArkIesInfo {
    int32_t photometric_type; /* 1 = C, 2 = B, 3 = A (IESProfile.h:25-29) */
    int32_t units_type;       /* 1 = feet, 2 = meters */
    int32_t lamp_count;
    uint32_t num_angles_v, num_angles_h;
    float lumens_per_lamp;
    float width, length, height;
    float ballast_factor, input_watts;
    float first_angle_v, last_angle_v, first_angle_h, last_angle_h;
    float max_candela;        /* after the candela multiplier */
} ArkIesInfo;

/* Parses `text` (length bytes, the .ies file contents) and writes the
 * lut_size x lut_size R32F table, row y = horizontal angle y/lut_size*360 deg,
 * column x = vertical angle x/lut_size*180 deg. out_info may be NULL. */
int ark_ies_lut_from_memory(const char* text, uint64_t length, uint32_t lut_size, float* out_lut, ArkIesInfo* out_info);

/* Same, reading the file at `path`. */
int ark_ies_lut_from_file(const char* path, uint32_t lut_size, float* out_lut, ArkIesInfo* out_info);

/* Candela value at (horizontal, vertical) degrees (IESProfile::lookupValue). */
int ark_ies_lookup(const char* text, uint64_t length, float angle_h, float angle_v, float* out_value);

/* Reason of the last failure on this thread ("" when none). */
const char* ark_ies_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* ARK_IES_H */
