/*
 * ark_scene.h — synthetic scene generators for the DDGI benchmark configs
 * (BASELINE.json configs C4/C5). The reference has no synthetic
 * scenes (Bistro/Sponza geometry is unavailable offline), so the benchmark
 * workload is a deterministic triangle-strip soup.
 *
 * The generated arrays are owned by the ArkSoupScene and exposed as a ready
 * ArkDdgiScene view (ark_soup_scene_view) for ark_ddgi_set_scene.
 */
#ifndef ARK_SCENE_H
#define ARK_SCENE_H

#include "ark_ddgi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ArkSoupParams {
    uint32_t struct_size;
    uint64_t triangle_count;   /* rounded down to a multiple of 16 (one strip = 16 triangles, 18 vertices) */
    float extent;              /* strip origins ~ U([0, extent]^3); default 31 */
    float step_min, step_max;  /* strip step length ~ U(step_min, step_max); default 0.05..0.3 */
    float width_min, width_max;/* strip width ~ U(width_min, width_max); default 0.05..0.3 */
    uint64_t seed;             /* PCG32 initstate; default 0xA2C05E00 */
    uint64_t stream;           /* PCG32 initseq; default 1 */
    uint32_t material_count;   /* default 16: one RT mesh + instance per material */
    float sun_color[3];        /* pre-exposed; default (3,3,3) */
    float sun_direction[3];    /* default normalize(0.5,-1,0.2) (ShowcaseApp.cpp:122) */
    int32_t has_sun;
} ArkSoupParams;

typedef struct ArkSoupScene ArkSoupScene;

/* Fills `p` with the defaults of BASELINE config C4 (10M triangles). */
void ark_soup_default_params(ArkSoupParams* p);
int ark_soup_generate(const ArkSoupParams* p, ArkSoupScene** out);
const ArkDdgiScene* ark_soup_scene_view(const ArkSoupScene* s);
void ark_soup_free(ArkSoupScene* s);

#ifdef __cplusplus
}
#endif

#endif /* ARK_SCENE_H */
