"""Host-side checks of the sync-free loss helpers (lpgnn.train / lpgnn.val)
against the oracle restatement of the reference (utils.py:286-299,
val.py:106-124, 199-237).  Runs on CPU tensors; the GPU twin is in
test_gpu_model.py."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O


@pytest.mark.parametrize("labels", [[0, 1, 2, 1, 1, 0], [1, 1, 2, 2, 2], [0, 0, 0], [1, 1], [2, 1, 2], [0, 2, 0]])
@pytest.mark.parametrize("merge", [True, False])
def test_balanced_weights_equal_reference(labels, merge):
    from lpgnn.train import labels_to_balanced_weights

    t = torch.tensor(labels, dtype=torch.int64)
    assert torch.equal(labels_to_balanced_weights(t, merge_lu=merge), O.labels_to_balanced_weights(t, merge_lu=merge))


def test_accuracy_device_formula_on_host():
    from lpgnn.val import accuracy, accuracy_device, inference_gnn

    rng = np.random.default_rng(2)
    m, n = 40, 60
    logits = torch.from_numpy(rng.standard_normal((m + n, 3)).astype(np.float32))
    gt = torch.from_numpy(rng.integers(0, 3, m + n))
    assert torch.equal(inference_gnn(logits, m), O.inference_gnn(logits, m))
    for a, b in zip(accuracy_device(logits, gt, m), accuracy(logits, gt, m, return_pr=True)):
        assert abs(a.item() - float(b)) < 1e-6
