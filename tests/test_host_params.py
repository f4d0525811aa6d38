"""Host-side parameter handling of the drop-in network (no GPU): tree_flatten order of the
leaves and the upload cache key of AINet.bind (tensor identity + in-place version)."""
import numpy as np
import torch

from aiqmc.wavefunction_Ynlm import nn


def test_flatten_matches_tree_flatten_order():
    tree = {"b": [torch.arange(3.0), torch.ones(2, 2)], "a": torch.tensor([7.0])}
    flat = nn.flatten_params(tree)
    assert flat.dtype == np.float64
    np.testing.assert_array_equal(flat, [7.0, 0.0, 1.0, 2.0, 1.0, 1.0, 1.0, 1.0])
    mixed = {"b": [np.arange(3.0), np.ones((2, 2))], "a": np.array([7.0])}
    np.testing.assert_array_equal(nn.flatten_params(mixed), flat)


def test_upload_key_tracks_identity_and_inplace_writes():
    leaves = nn.tree_leaves({"w": torch.zeros(4), "v": [torch.ones(2)]})
    key = nn._leaf_key(leaves)
    assert nn._same_leaves(key, leaves)
    leaves[0].add_(1.0)                       # in-place update: a new version
    assert not nn._same_leaves(key, leaves)
    key = nn._leaf_key(leaves)
    assert nn._same_leaves(key, leaves)
    other = [leaves[0].clone(), leaves[1]]    # same values, a different tensor
    assert not nn._same_leaves(key, other)
    assert nn._leaf_key([np.zeros(2)]) is None   # numpy leaves are compared by value
    assert not nn._same_leaves(None, leaves)
