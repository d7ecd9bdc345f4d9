"""lpgnn.options.PathOptions on CPU: the defaults, the LPGNN_* environment switches (read once, by
from_env), replace() and the arith check.  No kernels run."""
import pytest

from lpgnn.options import PathOptions

SWITCHES = {  # env name -> (field, value the switch selects)
    "LPGNN_FC_ARITH": ("arith", "fp32"),
    "LPGNN_REASSOC": ("reassociate", False),
    "LPGNN_FUSE_HEADS": ("fuse_heads", False),
    "LPGNN_FUSE_HEAD_FWD": ("fuse_head_fwd", False),
    "LPGNN_FOLD_RELU_BWD": ("fold_relu_bwd", False),
    "LPGNN_FOLD_CONV1_WGRAD": ("fold_conv1_wgrad", False),
    "LPGNN_OVERLAP": ("overlap", True),
    "LPGNN_RELU_BITS": ("relu_bits", False),
    "LPGNN_FOLD_BIAS_SUMS": ("fold_bias_sums", False),
    "LPGNN_SPMM_HEAVY": ("spmm_heavy", 256),
}


def _clear(monkeypatch):
    for k in SWITCHES:
        monkeypatch.delenv(k, raising=False)


def test_defaults_are_the_fused_f16x2_path(monkeypatch):
    _clear(monkeypatch)
    o = PathOptions.from_env()
    assert o == PathOptions()
    assert (o.arith, o.reassociate, o.fuse_heads, o.fuse_head_fwd, o.fold_relu_bwd, o.fold_conv1_wgrad,
            o.overlap, o.relu_bits, o.fold_bias_sums, o.spmm_heavy) == ("f16x2", True, True, True, True, True, False, True,
                                                                        True, 1024)


@pytest.mark.parametrize("name", sorted(SWITCHES))
def test_each_switch_sets_one_field(monkeypatch, name):
    _clear(monkeypatch)
    field, value = SWITCHES[name]
    raw = value if isinstance(value, str) else str(value) if type(value) is int else ("1" if value else "0")
    monkeypatch.setenv(name, raw)
    o = PathOptions.from_env()
    assert getattr(o, field) == value
    assert o.replace(**{field: getattr(PathOptions(), field)}) == PathOptions()


def test_replace_is_a_copy_and_arith_is_checked():
    base = PathOptions()
    alt = base.replace(fold_bias_sums=False)
    assert base.fold_bias_sums and not alt.fold_bias_sums
    with pytest.raises(ValueError):
        PathOptions(arith="fp64")
    with pytest.raises(Exception):
        base.relu_bits = False  # frozen: no module or object state a caller mutates


def test_spmm_heavy_default_matches_the_sparse_module():
    from lpgnn import sparse

    assert PathOptions().spmm_heavy == sparse.DEFAULT_HEAVY
    with pytest.raises(ValueError):
        PathOptions(spmm_heavy=-1)
