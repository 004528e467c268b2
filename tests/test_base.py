"""Host reduction kernel (transform2) for all dtypes x ops (parity: tests/cpp/unit/test_operations.cpp)."""
import numpy as np
import pytest
import torch

from kungfu_amd._lib import DTYPE_CODES, OP_CODES, runtime as K

DTYPES = [torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.float16, torch.bfloat16,
          torch.float32, torch.float64]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", ["sum", "min", "max", "prod"])
@pytest.mark.parametrize("n", [1, 7, 8, 33, 1000])
def test_transform2(dtype, op, n):
    g = torch.Generator().manual_seed(n)
    if dtype.is_floating_point:
        x = torch.randn(n, generator=g).to(dtype)
        y = torch.randn(n, generator=g).to(dtype)
    else:
        x = torch.randint(0, 5, (n,), generator=g).to(dtype)
        y = torch.randint(0, 5, (n,), generator=g).to(dtype)
    z = torch.empty_like(x)
    K.transform2(z.data_ptr(), x.data_ptr(), y.data_ptr(), n, DTYPE_CODES[dtype], OP_CODES[op])
    f = {"sum": torch.add, "min": torch.minimum, "max": torch.maximum, "prod": torch.mul}[op]
    if dtype in (torch.float16, torch.bfloat16):
        ref = f(x.float(), y.float()).to(dtype)
        torch.testing.assert_close(z.float(), ref.float(), rtol=0, atol=0)
    else:
        ref = f(x, y)
        assert torch.equal(z, ref)


def test_transform2_inplace_alias():
    x = torch.arange(100, dtype=torch.float32)
    y = torch.ones(100)
    K.transform2(x.data_ptr(), x.data_ptr(), y.data_ptr(), 100, DTYPE_CODES[torch.float32], 0)
    assert torch.equal(x, torch.arange(100, dtype=torch.float32) + 1)
