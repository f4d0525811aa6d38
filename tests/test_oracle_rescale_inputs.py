"""``make_ai_net(rescale_inputs=True)`` (wavefunction_Ynlm/nn.py:119-139, the branch at :126-131) in
the CPU oracle.  The rescaled e-e features are ee * log(1 + r_ee) / r_ee, and the reference masks
the r_ee diagonal to exactly 0 (nn.py:115), so each diagonal entry is (0 * 0) / 0 = NaN; the
g_two means of construct_symmetric_features (nn.py:151) carry it into every electron's features,
so the reference's log|psi| is NaN for every configuration.  The drop-in therefore refuses the
option (aiqmc/wavefunction_Ynlm/nn.py make_ai_net) instead of shipping kernels that return NaN;
this test pins that reading of the reference.  Parity unpinned beyond the restatement itself (no
JAX here to run the reference)."""
import numpy as np
import pytest
import torch

from oracle import network, system


@pytest.mark.parametrize("name", ["H2", "Be", "N2"])
def test_rescaled_inputs_give_nan_psi(name):
    s = system.make_system(name)
    p = network.to_torch(system.init_params(np.random.default_rng(3), s))
    pos = torch.tensor(system.init_electrons(np.random.default_rng(4), s.atoms, s.charges, 3, 1.0))
    plain = network.Network(s)
    resc = network.Network(s, rescale_inputs=True)
    for b in range(pos.shape[0]):
        assert torch.isfinite(plain.apply(p, pos[b])[1])
        assert torch.isnan(resc.apply(p, pos[b])[1])


def test_rescaled_features_nan_only_on_ee_diagonal():
    s = system.make_system("Be")
    pos = torch.tensor(system.init_electrons(np.random.default_rng(5), s.atoms, s.charges, 1, 1.0)[0])
    ae, ee, r_ae, r_ee = network.construct_input_features(pos, torch.tensor(s.atoms))
    lr_ee = torch.log(1 + r_ee)
    f = torch.cat([lr_ee, ee * lr_ee / r_ee], dim=2)
    diag = torch.eye(s.nelectrons, dtype=torch.bool)
    assert torch.isnan(f[diag][:, 1:]).all() and not torch.isnan(f[diag][:, 0]).any()
    assert torch.isfinite(f[~diag]).all()
    lr_ae = torch.log(1 + r_ae)
    assert torch.isfinite(torch.cat([lr_ae, ae * lr_ae / r_ae], dim=2)).all()


def test_drop_in_refuses_rescaled_inputs():
    from aiqmc.wavefunction_Ynlm import nn
    s = system.make_system("H2")
    t = s.tables()
    with pytest.raises(NotImplementedError, match="NaN"):
        nn.make_ai_net(s.nspins, s.charges, t["parallel_indices"], t["antiparallel_indices"],
                       t["spin_up_indices"], t["spin_down_indices"], t["parallel_indices"].shape[1],
                       t["antiparallel_indices"].shape[1], 3, s.natoms, s.nelectrons, rescale_inputs=True)
