"""resize_oracle.py — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).

numpy restatement of cv::resize(src, dst, Size(dW, dH), 0, 0, INTER_AREA) for integer downscale
factors as app/main.cpp:203 calls it on the grayscale frames: OpenCV 4.x's area-fast path
(modules/imgproc/src/resize.cpp resizeAreaFast_<uchar, int>): the fx·fy block sum (int) times the f32
reciprocal 1.f/(fx·fy), saturate_cast<uchar> = round half to even.  OpenCV is not in
/root/reference nor in this image: parity with it is unpinned; pinned here by closed forms (constant
blocks map to their value, a block of k ones and fx·fy−k zeros to round-half-even(k/(fx·fy)),
tests/test_dataset.py).
"""
import numpy as np


def resize_area(src, dW, dH):
    src = np.asarray(src, np.uint8)
    H, W = src.shape
    fx, fy = W // dW, H // dH
    assert fx * dW == W and fy * dH == H
    s = src.reshape(dH, fy, dW, fx).astype(np.int64).sum(axis=(1, 3))
    v = np.rint(s.astype(np.float32) * np.float32(1.0 / (fx * fy)))
    return np.clip(v, 0, 255).astype(np.uint8)
