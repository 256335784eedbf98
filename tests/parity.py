"""Shared comparison helpers for the parity tests."""
import numpy as np


def bit_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise f32 bit equality; any NaN equals any NaN (payloads differ by ISA)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def assert_bit_identical(gpu: np.ndarray, ref: np.ndarray, what: str = "") -> None:
    same = bit_equal(gpu, ref)
    if not same.all():
        idx = np.argwhere(~same)
        first = idx[:5].tolist()
        raise AssertionError(
            f"{what}: {(~same).sum()} of {same.size} f32 channels differ; first {first}: "
            f"gpu={[float(gpu[tuple(i)]) for i in idx[:5]]} ref={[float(ref[tuple(i)]) for i in idx[:5]]}"
        )
