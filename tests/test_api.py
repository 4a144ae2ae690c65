"""CPU: the drop-in's API surface matches the reference plugin (src/gaussian_renderer.py).

Ported from the reference's tests/test_gaussian_renderer.py (construction, factory, error
messages, background buffer); every check that needs pixels runs in test_reference_api_gpu.py
on the GPU, because the product has no CPU compute path (it raises a RuntimeError that
mentions CUDA, which the reference's own test accepts for 3D, :325-332).
"""
import pytest
import torch

from src.gaussian_renderer import (GaussianRenderer, GaussianRenderer2D, GaussianRenderer3D,
                                   convert_2d_to_3d_params, convert_3d_to_2d_params, create_renderer)


def test_cannot_instantiate_abstract():
    with pytest.raises(TypeError):
        GaussianRenderer(256, 256)


def test_subclass_must_implement_methods():
    class Incomplete(GaussianRenderer):
        pass
    with pytest.raises(TypeError):
        Incomplete(256, 256)


def test_2d_num_params_and_init():
    r = GaussianRenderer2D(256, 256, device="cpu")
    assert r.get_num_params() == 9
    assert (r.width, r.height, r.device) == (256, 256, "cpu")
    assert r.background_color.shape == (3,)
    assert (r.kernel_size, r.sigma_cutoff, r.batch_size) == (5, 3.0, 1)


def test_3d_num_params_and_init_without_gsplat():
    r = GaussianRenderer3D(256, 256, device="cpu")     # no ImportError: no gsplat dependency
    assert r.get_num_params() == 14
    assert (r.width, r.height, r.device) == (256, 256, "cpu")


def test_invalid_params_shape_messages():
    with pytest.raises(ValueError, match="Expected 9 parameters"):
        GaussianRenderer2D(64, 64, device="cpu").render(torch.randn(10, 14), None, None)
    with pytest.raises(ValueError, match="Expected 14 parameters"):
        GaussianRenderer3D(64, 64, device="cpu").render(torch.randn(10, 9), torch.eye(4), torch.eye(3))


def test_background_color_and_empty_scene():
    r = GaussianRenderer2D(32, 16, device="cpu")
    r.set_background_color(torch.tensor([0.0, 0.0, 1.0]))
    rgb, alpha = r.render(torch.zeros((0, 9)), None, None)
    assert rgb.shape == (16, 32, 3) and alpha.shape == (16, 32)
    assert torch.allclose(rgb[0, 0], torch.tensor([0.0, 0.0, 1.0]), atol=1e-5)
    assert float(alpha.abs().max()) == 0.0
    with pytest.raises(ValueError, match=r"Expected color shape \(3,\)"):
        r.set_background_color(torch.zeros(4))


def test_background_buffer_in_state_dict():
    r = create_renderer("3d", 8, 8, device="cpu")
    sd = r.state_dict()
    assert list(sd.keys()) == ["background_color"]      # checkpoints stay loadable


def test_factory():
    assert isinstance(create_renderer("2d", 256, 256, device="cpu"), GaussianRenderer2D)
    assert isinstance(create_renderer("3d", 256, 256, device="cpu"), GaussianRenderer3D)
    assert type(create_renderer("2d", 1, 1, device="cpu")) is type(create_renderer("2D", 1, 1, device="cpu"))
    with pytest.raises(ValueError, match="Unknown renderer mode"):
        create_renderer("invalid", 256, 256)
    r = create_renderer("2d", 256, 256, device="cpu", sigma_cutoff=4.0, kernel_size=7)
    assert r.sigma_cutoff == 4.0 and r.kernel_size == 7
    r3 = create_renderer("3d", 8, 8, device="cpu", sigma_cutoff=4.0)     # 3D drops the kwargs
    assert r3.radius_mode == "opacity_aabb"
    assert create_renderer("3d", 8, 8, device="cpu", radius_mode="isotropic_3sigma").radius_mode == "isotropic_3sigma"


def test_cpu_render_raises_runtime_error_mentioning_cuda():
    r3 = create_renderer("3d", 128, 96, device="cpu")
    with pytest.raises(RuntimeError, match="CUDA"):
        r3.render(torch.randn(10, 14), torch.eye(4), torch.eye(3))
    r2 = create_renderer("2d", 128, 96, device="cpu")
    with pytest.raises(RuntimeError, match="CUDA"):
        r2.render(torch.randn(10, 9), None, None)


def test_converters_not_implemented():
    with pytest.raises(NotImplementedError):
        convert_3d_to_2d_params(torch.zeros(1, 14), torch.eye(4), torch.eye(3))
    with pytest.raises(NotImplementedError):
        convert_2d_to_3d_params(torch.zeros(1, 9), torch.zeros(1), torch.eye(4), torch.eye(3))


def test_view_shard_covers_all_views():
    from gsr.multiview import view_shard
    for C in (1, 5, 6, 8, 13):
        for world in (1, 2, 3, 4, 8):
            got = []
            for r in range(world):
                sl = view_shard(C, world, r)
                got.extend(range(C)[sl])
            assert got == list(range(C))
            sizes = [len(range(C)[view_shard(C, world, r)]) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def test_background_cache_never_returns_stale_colour():
    """A freed background whose address is reused by a new tensor must not hit the cache."""
    from gsr.render import _background
    for _ in range(50):
        b1 = torch.tensor([0.1, 0.5, 0.9])
        assert torch.equal(_background(b1, 2, torch.device("cpu")), b1.expand(2, 3))
        del b1
        b2 = torch.ones(3)
        assert torch.equal(_background(b2, 2, torch.device("cpu")), torch.ones(2, 3))
        b2.mul_(0.5)                                   # in-place edit bumps the version
        assert torch.equal(_background(b2, 2, torch.device("cpu")), torch.full((2, 3), 0.5))
