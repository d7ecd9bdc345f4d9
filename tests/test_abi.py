"""The C-ABI library: builds for gfx950, loads, exports every declared symbol;
host pack (no GPU needed) equals the oracle's torch_sparse order."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import model_ref as O

HEADER = os.path.join(ROOT, "include", "lpgnn.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lpg_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from lpgnn import _lib

    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 8
    for name in names:
        assert hasattr(L, name), f"{name} declared in include/lpgnn.h but not exported"
    assert b"gfx950" in L.lpg_build_info()


def test_library_is_gfx950_code_object():
    from lpgnn import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_spmm_kernels_have_no_fused_multiply_add():
    """-ffp-contract=off is what makes the kernel bitwise equal to the CPU
    loop; guard it at the ISA level."""
    out = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "lp-gnn_amd"), "isa"], capture_output=True,
                         text=True)
    assert out.returncode == 0, out.stderr[-2000:]
    s = open("/tmp/lpg_isa/spmm-hip-amdgcn-amd-amdhsa-gfx950.s").read()
    assert "v_fma" not in s and "v_fmac" not in s and "v_pk_fma" not in s


def _coo(rng, m, n, nnz):
    keys = rng.choice(m * n, size=nnz, replace=False)
    return (keys // n).astype(np.int64), (keys % n).astype(np.int64), rng.uniform(-1, 1, nnz).astype(np.float32)


@pytest.mark.parametrize("m,n,nnz", [(5, 7, 0), (1, 1, 1), (64, 128, 700), (300, 50, 3000)])
def test_host_pack_matches_torch_sparse_order(m, n, nnz):
    from lpgnn import BipartiteCSR

    rng = np.random.default_rng(m * 31 + nnz)
    row, col, val = _coo(rng, m, n, nnz)
    adj = BipartiteCSR.from_coo(row, col, val, m, n, device="cpu")
    A = O.csr_from_coo(row, col, val, m, n)
    AT = O.csr_transpose(*A, m, n)
    for csr, ref in ((adj.fwd, A), (adj.bwd, AT)):
        assert np.array_equal(csr.rowptr.numpy(), ref[0])
        assert np.array_equal(csr.col.numpy(), ref[1])
        assert np.array_equal(csr.val.numpy(), ref[2])
    assert adj.t().sparse_sizes() == (n, m)


def test_host_pack_rejects_bad_input():
    from lpgnn import BipartiteCSR

    with pytest.raises(RuntimeError, match="duplicate edge"):
        BipartiteCSR.from_coo([0, 0], [1, 1], [0.5, 0.5], 2, 2, device="cpu")
    with pytest.raises(RuntimeError, match="out of"):
        BipartiteCSR.from_coo([0, 2], [1, 1], [0.5, 0.5], 2, 2, device="cpu")


def test_status_and_error_string():
    from lpgnn import _lib

    L = _lib.lib()
    empty = _lib.LpgCsr(0, 0, 0, None, None, None)  # valid and empty: the tuning check runs, no device work
    st = L.lpg_spmm_f32_tuned(ctypes.byref(empty), None, 0, None, 0, 0, None, 0, 0, 300, 0, None)
    assert st == 1
    assert b"slice_cols" in L.lpg_last_error()
    assert L.lpg_spmm_f32_tuned(ctypes.byref(empty), None, 0, None, 0, 0, None, 0, 0, 128, 16, None) == 0
    assert L.lpg_spmm_f32_tuned(ctypes.byref(empty), None, 0, None, 0, 0, None, 0, 0, 0, 7, None) == 1
    # an FC kernel choice past the entry's range is rejected before any launch (the pointers are
    # never dereferenced: the flags check precedes every device call)
    fake = 1 << 20
    assert L.lpg_fc_bf16(1, 8, 64, fake, 64, fake, 64, 0, None, 0, None, 0, None, fake, 8, _lib.fc_kernel(9), 0.0, 0,
                         0, None, None) == 1
    assert b"flags" in L.lpg_last_error()
    # NULL CSR -> invalid argument, no device work
    assert L.lpg_spmm_f32(None, None, 0, None, 0, 0, None) == 1
    assert L.lpg_csr_pack_workspace_bytes(-1, 0, 0) == -1


def test_no_cpu_path_for_spmm():
    from lpgnn import BipartiteCSR, spmm

    adj = BipartiteCSR.from_coo([0, 1], [1, 0], [0.5, -0.5], 2, 2, device="cpu")
    with pytest.raises(RuntimeError, match="no CPU path"):
        spmm(adj, torch.ones(2, 4))


def test_spmm_sum_op_registered_with_torch_sparse_schema():
    """torch.ops.lpgnn.spmm_sum takes torch_sparse 0.6.12's spmm_sum
    arguments (row, rowptr, col, value, colptr, csr2csc, mat) and has no CPU
    path."""
    import lpgnn  # noqa: F401  (registers the op)

    schema = str(torch.ops.lpgnn.spmm_sum.default._schema)
    assert "Tensor? row, Tensor rowptr, Tensor col, Tensor? value, Tensor? colptr, Tensor? csr2csc, Tensor mat" \
        in schema, schema
    rowptr = torch.tensor([0, 1, 2])
    col = torch.tensor([1, 0])
    with pytest.raises(RuntimeError, match="no CPU path"):
        torch.ops.lpgnn.spmm_sum(None, rowptr, col, None, None, None, torch.ones(2, 4))


def test_fc_rejects_unpadded_k_on_the_tiled_path():
    """lpg_fc_f32's tiled kernel needs K1, K2 multiples of 32 (the host pads);
    the check fails before any device work."""
    from lpgnn import _lib

    L = _lib.lib()
    fake = 1 << 20  # 16-byte aligned, never dereferenced: validation fails first
    st = L.lpg_fc_f32(10, 64, 40, fake, 40, fake, 40, 0, None, 0, None, 0, None, fake, 64, 0, 0.0, 0, 0, None, None)
    assert st == 1 and b"multiples of 32" in L.lpg_last_error()


def test_no_shipped_kernel_uses_scratch():
    """The spill rule: no kernel of ours in the shipped library uses scratch.  A
    register-spilling bf16 FC tile once gave wrong bits -- hipcc's spill code dropped the last
    dword of a partially reused accumulator tuple -- so spilling kernels are not shipped at all."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_resources as KR
    from lpgnn import _lib

    rows = KR.kernels(_lib.LIB_PATH)
    ours = [(n, s) for n, _, s in rows if KR.is_ours(n)]
    assert len(ours) > 50, len(ours)
    assert [n for n, s in ours if s] == []
