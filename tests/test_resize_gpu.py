"""GPU parity of erp_resize_area (csrc/resize.hip) against oracle/resize_oracle.py — bitwise.
cv::resize(..., INTER_AREA) of the frames (app/main.cpp:203), integer factors."""
import numpy as np
import pytest

from test_dataset import load_resize_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(vio):
    c = vio.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("W,H,dW,dH", [(3840, 1920, 960, 480), (960, 480, 480, 240), (90, 60, 30, 20),
                                       (64, 48, 64, 48), (100, 40, 20, 8)])
def test_bitwise_vs_oracle(ctx, W, H, dW, dH):
    ro = load_resize_oracle()
    rng = np.random.default_rng(W + H)
    img = rng.integers(0, 256, (H, W), dtype=np.uint8)
    np.testing.assert_array_equal(ctx.resize_area(img, dW, dH), ro.resize_area(img, dW, dH))


def test_erp_frame_and_strided_source(ctx, synth):
    ro = load_resize_oracle()
    f = synth.render_erp(3840, 1920, seed=3, rows_per_chunk=256)
    np.testing.assert_array_equal(ctx.resize_area(f, 960, 480), ro.resize_area(f, 960, 480))
    big = np.zeros((480, 1000), np.uint8)
    big[:, :960] = np.random.default_rng(1).integers(0, 256, (480, 960))
    view = big[:, :960]  # row stride 1000: not 16-byte aligned rows
    np.testing.assert_array_equal(ctx.resize_area(view, 240, 120), ro.resize_area(view, 240, 120))


def test_factor2_rounds_half_up(ctx):
    """2x2 blocks follow OpenCV's ResizeAreaFastVec, (a + b + c + d + 2) >> 2: {1,1,0,0} -> 1 (round
    half up), not the half-to-even 0 of the generic area-fast formula."""
    blocks = np.array([[1, 1, 0, 0], [1, 0, 0, 0], [3, 3, 0, 0], [1, 1, 1, 0]], np.uint8)
    img = np.zeros((2, 8), np.uint8)
    for i, b in enumerate(blocks):
        img[:, 2 * i:2 * i + 2] = b.reshape(2, 2)
    np.testing.assert_array_equal(ctx.resize_area(img, 4, 1)[0], [1, 0, 2, 1])


def test_non_integer_factor_rejected(vio, ctx):
    with pytest.raises(vio.VioError):
        ctx.resize_area(np.zeros((480, 960), np.uint8), 640, 320)


def test_device_batched_frames(ctx):
    torch = pytest.importorskip("torch")
    ro = load_resize_oracle()
    rng = np.random.default_rng(7)
    frames = rng.integers(0, 256, (3, 480, 960), dtype=np.uint8)
    d_src = torch.from_numpy(frames).to("cuda:0")
    d_dst = torch.zeros((3, 120, 240), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    ctx.resize_area_device(d_src.data_ptr(), 960, 480, 960, 3, d_dst.data_ptr(), 240, 120, 240)
    assert ctx.resize_kernel_ms() > 0
    out = d_dst.cpu().numpy()
    for f in range(3):
        np.testing.assert_array_equal(out[f], ro.resize_area(frames[f], 240, 120))
