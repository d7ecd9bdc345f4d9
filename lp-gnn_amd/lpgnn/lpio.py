"""On-disk LP format and node features -- host side.

The reference stores one LP per msgpack file (utils.py:193-224) with numpy
arrays encoded by ``msgpack_numpy`` (upstream, not installed here: its ext
format -- a map {b'nd': True, b'type': dtype.str, b'kind': b'', b'shape',
b'data': raw bytes} -- is restated below), in two layouts:

* raw  (scripts/cvt_to_pkl.py:262-265):
  [c, b_l, (row, col, data), b_u, l, u, con_lbls, var_lbls, con_nms, var_nms]
* processed (dataset.py:213-217):
  [row, col, A_data, c_feas, v_feas, y_s, y_t, ncons + nvars]

``process_raw`` is LPDataset.process for one file (dataset.py:178-224):
``scaling`` (dataset.py:23-76) + ``cvt_to_features`` (dataset.py:79-96) with
the utils.py helpers (323-383) and the label/bound checks (dataset.py:201-207).
This is data preparation, not the GPU hot path; it runs on the host.
"""
from __future__ import annotations

import logging

import numpy as np
import scipy.sparse as sp


# ------------------------------------------------------------ msgpack I/O
def np_encode(obj):
    """msgpack_numpy.encode (ndarray / numpy scalar -> map)."""
    if isinstance(obj, np.ndarray):
        if obj.dtype.kind == "V":
            kind, descr = b"V", obj.dtype.descr
        else:
            kind, descr = b"", obj.dtype.str
        return {b"nd": True, b"type": descr, b"kind": kind, b"shape": obj.shape,
                b"data": np.ascontiguousarray(obj).tobytes()}
    if isinstance(obj, (np.bool_, np.number)):
        return {b"nd": False, b"type": obj.dtype.str, b"data": obj.tobytes()}
    if isinstance(obj, complex):
        return {b"complex": True, b"data": repr(obj)}
    return obj


def _dtype(descr):
    if isinstance(descr, (str, bytes)):
        return np.dtype(descr.decode() if isinstance(descr, bytes) else descr)
    return np.dtype([tuple(t.decode() if isinstance(t, bytes) else t for t in d) for d in descr])


def np_decode(obj):
    """msgpack_numpy.decode (map -> ndarray / numpy scalar)."""
    try:
        if b"nd" in obj:
            if obj[b"nd"] is True:
                return np.ndarray(buffer=obj[b"data"], dtype=_dtype(obj[b"type"]), shape=obj[b"shape"]).copy()
            return np.frombuffer(obj[b"data"], dtype=_dtype(obj[b"type"]))[0]
        if b"complex" in obj:
            d = obj[b"data"]
            return complex(d.decode() if isinstance(d, bytes) else d)
    except (KeyError, TypeError):
        pass
    return obj


def msgpack_dump(obj, path) -> None:
    """utils.py:193-200."""
    import msgpack

    with open(str(path), "wb") as fp:
        msgpack.pack(obj, fp, default=np_encode, use_bin_type=True)


def msgpack_load(path):
    """utils.py:203-224 (object_hook = msgpack_numpy.decode, lists, str keys)."""
    import msgpack

    with open(str(path), "rb") as fp:
        return msgpack.unpack(fp, object_hook=np_decode, use_list=True, raw=False, strict_map_key=False)


# --------------------------------------------------------- feature helpers
def sparse_mat_div_by_vec(A, vec, axis="row"):
    """utils.py:323-332."""
    vec = np.asarray(vec).flatten()
    if axis == "row":
        B = A.tocsr(copy=True)
        B.data /= np.repeat(vec, B.getnnz(axis=1))
        return B
    B = A.tocsc(copy=True)
    B.data /= np.repeat(vec, B.getnnz(axis=0))
    return B


def count_nonzero_sparse_mat(A, by="col"):
    """utils.py:335-347."""
    nrows, ncols = A.shape
    row, col = A.nonzero()
    if by == "col":
        nnz = np.zeros(ncols)
        idx, cnts = np.unique(col, return_counts=True)
    else:
        nnz = np.zeros(nrows)
        idx, cnts = np.unique(row, return_counts=True)
    nnz[idx] = cnts
    return nnz


def cos_sim_vec_and_sparse_mat(v, A, bound=1e8):
    """utils.py:350-362."""
    v = np.clip(np.asarray(v), -bound, bound)
    nrm_b = np.sqrt((v ** 2).sum())
    nrm_cols = np.array(np.sqrt((A.multiply(A)).sum(0))).flatten()
    dot = v * A
    assert (dot[nrm_cols == 0] == 0).all()
    nrm_cols[nrm_cols == 0] = 1e-6
    if nrm_b == 0:
        nrm_b = 1e-6
    return dot / (nrm_b * nrm_cols)


def cos_sim_sparse_mat_and_vec(A, v, bound=1e8):
    """utils.py:365-366."""
    return cos_sim_vec_and_sparse_mat(v, A.T, bound)


def expand_inf(x):
    """utils.py:369-375: (value, tag) with tag +1 for +inf, -1 for -inf, value 0 there."""
    ori = np.array(x, copy=True)
    tag = np.zeros_like(ori)
    tag[ori == np.inf] = 1
    tag[ori == -np.inf] = -1
    ori[np.abs(ori) == np.inf] = 0
    return np.stack((ori, tag), axis=1)


def concatenate_on_lst_dim(*args):
    """utils.py:378-384."""
    return np.concatenate([a.reshape(-1, 1) if a.ndim == 1 else a for a in args], axis=1)


# ------------------------------------------------------------------ scaling
def scaling(c, b_l, A, b_u, l, u):
    """dataset.py:23-76: row scaling by the bounds, column scaling by |A| and
    the variable bounds, objective normalised to max |c| = 1."""
    b_u[b_u > 1e308] = np.inf
    b_l[b_l < -1e308] = -np.inf
    u[u > 1e308] = np.inf
    l[l < -1e308] = -np.inf

    scale_l = np.abs(b_l)
    scale_l[(scale_l == np.inf) | (scale_l == 0)] = 1
    scale_u = np.abs(b_u)
    scale_u[(scale_u == np.inf) | (scale_u == 0)] = 1
    scale_row = np.maximum(scale_l, scale_u)
    A = sparse_mat_div_by_vec(A, scale_row, "row")
    b_l /= scale_row
    b_u /= scale_row

    scale_l = np.abs(l)
    scale_l[(scale_l == np.inf) | (scale_l == 0)] = 1
    scale_u = np.abs(u)
    scale_u[(scale_u == np.inf) | (scale_u == 0)] = 1
    scale_col2 = np.maximum(1. / scale_l, 1. / scale_u)
    scale_col = np.abs(A).max(0).toarray().flatten()
    scale_col[(scale_col == np.inf) | (scale_col == 0)] = 1
    scale_col = np.maximum(scale_col, scale_col2)

    A = sparse_mat_div_by_vec(A, scale_col, "col")
    A = A.tocsr()
    l *= scale_col
    u *= scale_col
    c = c / scale_col
    scale_c = np.abs(c).max()
    if scale_c == 0.:
        logging.warning("all c is zero: feasibility problem?")
        scale_c = 1.
    c /= scale_c
    return c, b_l, A, b_u, l, u


def cvt_to_features(c, b_l, A, b_u, l, u):
    """dataset.py:79-96 -> (v_features [n, 8], c_features [m, 8])."""
    nrows, ncols = A.shape
    v_features = concatenate_on_lst_dim(
        c, count_nonzero_sparse_mat(A, "col") / nrows, cos_sim_vec_and_sparse_mat(b_l, A),
        cos_sim_vec_and_sparse_mat(b_u, A), expand_inf(l), expand_inf(u))
    c_features = concatenate_on_lst_dim(
        cos_sim_sparse_mat_and_vec(A, c), count_nonzero_sparse_mat(A, "row") / ncols,
        cos_sim_sparse_mat_and_vec(A, l), cos_sim_sparse_mat_and_vec(A, u), expand_inf(b_l), expand_inf(b_u))
    return v_features, c_features


def process_raw(raw):
    """LPDataset.process for one raw record (dataset.py:188-217) ->
    the processed record [row, col, A_data, c_feas, v_feas, y_s, y_t, nnodes]."""
    c, b_l, (row, col, data), b_u, l, u, con_lbls, var_lbls, con_nms, var_nms = raw
    c, b_l, b_u, l, u = (np.array(x, dtype=np.float64, copy=True) for x in (c, b_l, b_u, l, u))
    ncons, nvars = len(con_nms), len(var_nms)
    A = sp.coo_matrix((np.asarray(data, np.float64), (np.asarray(row), np.asarray(col))),
                      shape=(ncons, nvars)).tocsr()
    c, b_l, A, b_u, l, u = scaling(c, b_l, A, b_u, l, u)
    ncons, nvars = A.shape
    v_feas, c_feas = cvt_to_features(c, b_l, A, b_u, l, u)
    v_feas, c_feas = v_feas.astype(np.float32), c_feas.astype(np.float32)
    y_s, y_t = np.asarray(con_lbls, np.int64), np.asarray(var_lbls, np.int64)
    cons_l, cons_u = c_feas[:, -3] != 0, c_feas[:, -1] != 0
    vars_l, vars_u = v_feas[:, -3] != 0, v_feas[:, -1] != 0
    assert (y_s[cons_l] != 0).all()
    assert (y_s[cons_u] != 2).all()
    violates = int((y_t[vars_l] == 0).sum())
    if violates:
        logging.warning(f"violate {violates}")
    assert (y_t[vars_u] != 2).all()
    A = A.tocoo()
    return [A.row, A.col, A.data, c_feas, v_feas, y_s, y_t, ncons + nvars]


def load_processed(path, device="cpu", thresh_num=np.inf, record=None):
    """LPDataset.get (dataset.py:229-264) + MyToBipartite (268-332) for one
    processed file -> a BipartiteBatch with the dual CSR packed on `device`.
    ``record``: the file's already-decoded msgpack record (no second read)."""
    from .data import MyToBipartite, lp_to_unipartite

    row, col, A_data, c_feas, v_feas, y_s, y_t, nnodes = msgpack_load(path) if record is None else record
    data = lp_to_unipartite(row, col, A_data, c_feas, v_feas, y_s, y_t, processed_path=str(path))
    assert data.num_nodes == int(nnodes)
    return MyToBipartite(dev=device, thresh_num=thresh_num)(data)


def load_bipartite(path, device="cpu", record=None):
    """load_processed without the to_undirected / split round trip: the .pk
    record straight to a BipartiteBatch (data.bipartite_from_lp)."""
    from .data import bipartite_from_lp

    row, col, A_data, c_feas, v_feas, y_s, y_t, nnodes = msgpack_load(path) if record is None else record
    assert int(nnodes) == np.asarray(c_feas).shape[0] + np.asarray(v_feas).shape[0]
    return bipartite_from_lp(row, col, A_data, c_feas, v_feas, y_s, y_t, device, processed_path=str(path))
