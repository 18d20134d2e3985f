"""CPU oracle of the DDGI consumer, lightingCompose.comp:22-135,
against closed forms. The reference ships no fixtures for this shader: parity
unpinned against the Vulkan driver; the HIP kernel is checked bit for bit against
this restatement in test_gpu_compose.py."""
import numpy as np

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
import compose_inputs as CI
import oracle_lib as O
from parity import make_desc

W, H = 24, 16


def _oracle():
    grid = D.ProbeGrid((4, 3, 4), (0.7, 0.7, 0.7), (-1.0, 0.0, -1.0))
    cfg = D.DDGIConfig(rays_per_probe=16, probe_updates_per_frame=48, max_rays_per_probe=16, max_probe_updates=48)
    return O.Oracle(make_desc(grid, 100.0, cfg))


def _uniform_irradiance(o, value):
    irr = o.read(abi.ARK_DDGI_ATLAS_IRRADIANCE).reshape(-1, 4)
    irr[:] = O.f32_to_f16(np.full(4, value, np.float32))
    o.write(abi.ARK_DDGI_ATLAS_IRRADIANCE, irr.reshape(-1))


def test_sky_pixels_pass_direct_light_through():
    """depth >= 1 - 1e-6: only direct light (+ skin diffuse) reach the output (:56-70)."""
    o = _oracle()
    g = CI.gbuffer(W, H, sky_frac=1.0)
    cam = CI.camera(W, H)
    out = o.lighting_compose(W, H, abi.ARK_COMPOSE_DIRECT_LIGHT | abi.ARK_COMPOSE_DIFFUSE_GI | abi.ARK_COMPOSE_GLOSSY_GI, cam, g)
    assert np.array_equal(out, g["direct_light"])
    out = o.lighting_compose(W, H, abi.ARK_COMPOSE_SKIN_DIFFUSE_LIGHT, cam, g)  # materialBaseColor = 1
    di = O.f16_to_f32(g["diffuse_irradiance"])[..., :3].astype(np.float64) / np.pi
    assert np.allclose(O.f16_to_f32(out)[..., :3], di, rtol=2e-3, atol=1e-6)
    assert (out[..., 3] == 0).all()
    o.close()


def test_uniform_atlas_closed_form():
    """All irradiance texels = a: every probe gives a^2.5, so the DDGI term is
    (a^2.5)^2 * pi/2 = a^5 pi/2 whatever the weights; with no reflections the
    colour is baseColor * a^5 pi/2 * ao, ao = min(ssao, baked occlusion)."""
    o = _oracle()
    a = 0.75
    _uniform_irradiance(o, a)
    g = CI.gbuffer(W, H, sky_frac=0.0, reflect_frac=0.0)
    flags = (abi.ARK_COMPOSE_DIFFUSE_GI | abi.ARK_COMPOSE_MATERIAL_COLOR | abi.ARK_COMPOSE_BAKED_OCCLUSION
             | abi.ARK_COMPOSE_SCREEN_SPACE_OCCLUSION)
    out = O.f16_to_f32(o.lighting_compose(W, H, flags, CI.camera(W, H), g))
    bc = g["base_color"][..., :3].astype(np.float64) / 255
    ao = np.minimum(g["screen_space_occlusion"], g["material"][..., 2] / 255.0)[..., None]
    want = bc * (a ** 5) * np.pi / 2 * ao
    assert np.allclose(out[..., :3], want, rtol=3e-3, atol=1e-5)
    # bent normals: ao also takes min with |bent normal| where the cone is >= 0
    out2 = O.f16_to_f32(o.lighting_compose(W, H, flags | abi.ARK_COMPOSE_USE_BENT_NORMAL | abi.ARK_COMPOSE_BENT_NORMAL_OCCLUSION,
                                           CI.camera(W, H), g))
    bn = O.f16_to_f32(g["bent_normal"]).astype(np.float64)
    blen = np.linalg.norm(bn[..., :3], axis=-1)
    ao2 = np.where(bn[..., 3] >= 0, np.minimum(ao[..., 0], blen), ao[..., 0])[..., None]
    assert np.allclose(out2[..., :3], bc * (a ** 5) * np.pi / 2 * ao2, rtol=3e-3, atol=1e-5)
    o.close()


def test_glossy_and_fudge_factor():
    """With a reflection direction: + baseColor * reflections * 0.25 (:95-99) and the
    DDGI term scaled by (1 - metallic)(1 - F); without: no glossy term, full diffuse."""
    o = _oracle()
    _uniform_irradiance(o, 0.0)  # DDGI term 0: only the glossy term remains
    g = CI.gbuffer(W, H, sky_frac=0.0, reflect_frac=0.5)
    out = O.f16_to_f32(o.lighting_compose(W, H, abi.ARK_COMPOSE_GLOSSY_GI | abi.ARK_COMPOSE_DIFFUSE_GI | abi.ARK_COMPOSE_MATERIAL_COLOR,
                                          CI.camera(W, H), g))
    has = np.linalg.norm(O.f16_to_f32(g["reflection_direction"])[..., :3].astype(np.float64), axis=-1) ** 2 > 1e-4
    bc = g["base_color"][..., :3].astype(np.float64) / 255
    refl = O.f16_to_f32(g["reflections"])[..., :3].astype(np.float64)
    want = np.where(has[..., None], bc * refl * 0.25, 0.0)
    assert np.allclose(out[..., :3], want, rtol=2e-3, atol=1e-6)
    o.close()


def test_threads_do_not_change_bits():
    o = _oracle()
    _uniform_irradiance(o, 0.4)
    g = CI.gbuffer(W, H)
    cam = CI.camera(W, H)
    a = o.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, g, threads=1)
    b = o.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, g, threads=5)
    assert np.array_equal(a, b)
    o.close()
