"""Input transforms (VIT:32-46): the CPU oracle pinned on Pillow, the host-side
parameter draw, and (-m gpu) the HIP resample kernels bit-exact against the oracle and Pillow."""
import os

import numpy as np
import pytest
import torch

from oracle import image_ref as O

DEV = "cuda"


def test_oracle_matches_pillow_fixture(golden_dir):
    fx = np.load(os.path.join(golden_dir, "image_golden.npz"))
    n = sum(1 for k in fx.files if k.startswith("in"))
    assert n >= 8
    for i in range(n):
        img, want = fx[f"in{i}"], fx[f"out{i}"]
        got = O.resize_u8(img, want.shape[0], want.shape[1])
        assert np.array_equal(got, want), i


@pytest.mark.parametrize("h,w,oh,ow", [(375, 500, 224, 224), (300, 17, 224, 224), (13, 900, 224, 224),
                                       (500, 333, 256, 384), (224, 224, 224, 224), (2, 3, 224, 224)])
def test_oracle_matches_live_pillow(h, w, oh, ow):
    from PIL import Image
    img = np.random.default_rng(h * 7 + w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    want = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    assert np.array_equal(O.resize_u8(img, oh, ow), want)


def test_oracle_train_and_val_chains_match_pillow():
    """crop -> resize -> flip -> ToTensor -> Normalize, and Resize(256) -> CenterCrop(224), as torchvision
    composes them on PIL images (restated: torchvision is absent)."""
    from PIL import Image
    img = np.random.default_rng(5).integers(0, 256, (341, 460, 3), dtype=np.uint8)
    pil = Image.fromarray(img)
    top, left, h, w = 17, 40, 200, 310
    r = np.asarray(pil.crop((left, top, left + w, top + h)).resize((224, 224), Image.BILINEAR))
    r = r[:, ::-1]
    want = (np.transpose(r, (2, 0, 1)).astype(np.float32) / np.float32(255) - O.MEAN[:, None, None]) / O.STD[:, None, None]
    assert np.array_equal(O.train_transform(img, top, left, h, w, True), want)
    rh, rw = O.resize_shorter(341, 460)
    assert (rh, rw) == (256, 345)
    v = np.asarray(pil.resize((rw, rh), Image.BILINEAR))
    t, l_ = int(round((rh - 224) / 2.0)), int(round((rw - 224) / 2.0))
    v = v[t:t + 224, l_:l_ + 224]
    want = (np.transpose(v, (2, 0, 1)).astype(np.float32) / np.float32(255) - O.MEAN[:, None, None]) / O.STD[:, None, None]
    assert np.array_equal(O.val_transform(img), want)


def test_random_resized_crop_params_in_bounds_and_seeded():
    from vit_amd import data
    g = torch.Generator().manual_seed(0)
    seen = set()
    for H, W in [(375, 500), (500, 375), (20, 1000), (1000, 20), (224, 224), (1, 1)]:
        for _ in range(50):
            t, l_, h, w = data.random_resized_crop_params(H, W, g)
            assert 0 <= t and 0 <= l_ and 0 < h and 0 < w and t + h <= H and l_ + w <= W
            seen.add((H, W, h, w))
    assert len(seen) > 100
    a = data.random_resized_crop_params(375, 500, torch.Generator().manual_seed(3))
    b = data.random_resized_crop_params(375, 500, torch.Generator().manual_seed(3))
    assert a == b
    # extreme aspect ratio never satisfies the ratio bounds: central-crop fallback
    assert data.random_resized_crop_params(1000, 20, torch.Generator().manual_seed(1))[3] == 20


def test_plan_validates_and_lays_out_batch():
    from vit_amd import data
    tr = data.GpuTransform(train=True, device="cpu")
    tab = tr.plan([(100, 80), (50, 60)], params=[(0, 0, 100, 80, False), (10, 5, 40, 55, True)])
    assert tab.shape == (2, 12)
    assert list(tab[1][:3]) == [100 * 80 * 3, 60, 10] and tab[1][10] == 1 and tab[1][11] == 100 * 224 * 3
    with pytest.raises(ValueError):
        tr.plan([(10, 10)], params=[(5, 0, 6, 10, False)])
    va = data.GpuTransform(train=False, device="cpu")
    tab = va.plan([(341, 460)])
    assert list(tab[0][6:10]) == [256, 345, 16, 60]
    with pytest.raises(ValueError):
        data.GpuTransform(train=False, resize=200, device="cpu").plan([(300, 300)])


# ------------------------------------------------------------------------------------------ GPU

def _images(shapes, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]


@pytest.mark.gpu
def test_gpu_train_transform_bit_exact():
    from vit_amd import data
    shapes = [(375, 500), (500, 375), (64, 48), (224, 224), (1200, 900), (30, 700), (1, 1)]
    imgs = _images(shapes, 1)
    tr = data.GpuTransform(train=True)
    g = torch.Generator().manual_seed(42)
    params = tr.draw(shapes, g)
    # include a full-image crop and a 1-pixel-wide crop
    params[2] = (0, 0, 64, 48, True)
    params[5] = (3, 10, 20, 1, False)
    out = tr(imgs, params=params).cpu().numpy()
    torch.cuda.synchronize()
    for b, (img, (t, l_, h, w, f)) in enumerate(zip(imgs, params)):
        want = O.train_transform(img, t, l_, h, w, f)
        assert np.array_equal(out[b], want), (b, np.abs(out[b] - want).max())


@pytest.mark.gpu
def test_gpu_train_transform_random_draw_matches_pillow():
    """The generator-driven path end to end against Pillow itself."""
    from PIL import Image
    from vit_amd import data
    shapes = [(333, 500), (480, 640)]
    imgs = _images(shapes, 2)
    tr = data.GpuTransform(train=True)
    out = tr(imgs, generator=torch.Generator().manual_seed(9)).cpu().numpy()
    params = tr.draw(shapes, torch.Generator().manual_seed(9))
    for b, (img, (t, l_, h, w, f)) in enumerate(zip(imgs, params)):
        r = np.asarray(Image.fromarray(img).crop((l_, t, l_ + w, t + h)).resize((224, 224), Image.BILINEAR))
        if f:
            r = r[:, ::-1]
        want = (np.transpose(r, (2, 0, 1)).astype(np.float32) / np.float32(255) - O.MEAN[:, None, None]) / O.STD[:, None, None]
        assert np.array_equal(out[b], want), b


@pytest.mark.gpu
def test_gpu_val_transform_bit_exact():
    from vit_amd import data
    shapes = [(375, 500), (500, 375), (256, 256), (341, 460), (2000, 300)]
    imgs = _images(shapes, 3)
    out = data.GpuTransform(train=False)(imgs).cpu().numpy()
    for b, img in enumerate(imgs):
        assert np.array_equal(out[b], O.val_transform(img)), b


@pytest.mark.gpu
def test_gpu_transform_empty_batch_and_feeds_model():
    import vit_amd
    from vit_amd import data
    assert data.GpuTransform(train=True)([]).shape == (0, 3, 224, 224)
    x = data.GpuTransform(train=True)(_images([(300, 400)] * 2, 4), generator=torch.Generator().manual_seed(0))
    m = vit_amd.create_model("vit_base_patch16_224").to(DEV)
    assert m(x).shape == (2, 1000)
