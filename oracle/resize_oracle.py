"""resize_oracle.py — TEST INFRASTRUCTURE ONLY (parity checker, never shipped).

numpy restatement of cv::resize(src, dst, Size(dW, dH), 0, 0, INTER_AREA) for integer downscale
factors as app/main.cpp:203 calls it on the grayscale frames: OpenCV 4.x's area-fast path
(modules/imgproc/src/resize.cpp resizeAreaFast_<uchar, int>): the fx·fy block sum (int) times the f32
reciprocal 1.f/(fx·fy), saturate_cast<uchar> = round half to even — except for fx = fy = 2, where
OpenCV's ResizeAreaFastVec (the only vectorised area-fast case for 1-channel u8) computes
(a + b + c + d + 2) >> 2, i.e. round half UP.  OpenCV is not in
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
    if fx == 2 and fy == 2:  # ResizeAreaFastVec: (sum + 2) >> 2
        return ((s + 2) >> 2).astype(np.uint8)
    v = np.rint(s.astype(np.float32) * np.float32(1.0 / (fx * fy)))
    return np.clip(v, 0, 255).astype(np.uint8)
