"""bqsr_copy_async (include/adam_bqsr.h): the kernel copy the streamed path
uses for its D2H, on aligned and unaligned buffers of every size class --
every byte checked (the tail bytes of an unaligned buffer are copied by a
grid-stride loop over a capped grid)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes,off_src,off_dst", [(1, 0, 0), (17, 0, 0), (100_003, 1, 0), (100_000, 0, 3),
                                                    (3 << 20, 5, 7), ((8 << 20) + 9, 0, 0)])
@pytest.mark.parametrize("host_dst", [False, True])
def test_copy_async_every_byte(nbytes, off_src, off_dst, host_dst):
    import torch
    from adam_amd import _capi, bqsr
    L = _capi.lib()
    ctx = bqsr.Context.get(0)
    g = torch.Generator().manual_seed(nbytes)
    src_h = torch.randint(0, 256, (nbytes + off_src,), dtype=torch.uint8, generator=g)
    src = src_h.cuda()
    if host_dst:
        dst = torch.zeros(nbytes + off_dst + 64, dtype=torch.uint8, pin_memory=True)
    else:
        dst = torch.zeros(nbytes + off_dst + 64, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    _capi.check(L.bqsr_copy_async(ctx.handle, ctypes.c_void_p(dst.data_ptr() + off_dst),
                                  ctypes.c_void_p(src.data_ptr() + off_src), nbytes, ctypes.c_void_p(st.cuda_stream)))
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    want = src_h.numpy()[off_src:]
    assert np.array_equal(got[off_dst:off_dst + nbytes], want)
    assert not got[:off_dst].any() and not got[off_dst + nbytes:].any()
