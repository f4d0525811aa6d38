"""CPU oracle for the AIQMC VMC hot path -- TEST INFRASTRUCTURE ONLY.

This package is a float64 CPU restatement of the reference algorithms on the
hot path (``AIQMCrelease3`` wavefunction forward, local energy, Metropolis
step).  It exists to check the HIP kernels; it is never imported by the
product package (``aiqmc``), and only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may use it.

Modules
-------
system      spin/pair index tables, walker initialisation, parameter init,
            canonical parameter flattening (tree_flatten order)
network     torch float64 restatement of ``wavefunction_Ynlm/nn.py`` (+ blocks,
            Jastrow, envelope), differentiable with torch.func
network_np  independent numpy restatement of the forward pass (value only)
hamiltonian potentials + kinetic energy via jvp-of-grad (the reference's
            ``Energy/hamiltonian.py:100-131`` algorithm) and via Hessian trace
mcstep      ``VMC/VMCmcstep.py`` walkers_update with host-injected randoms

Pinning status (see DESIGN.md "Oracle")
---------------------------------------
* The generic local-energy machinery (jvp-of-grad Laplacian, potentials,
  slogdet) is pinned by the known-answer tests the reference's own vendored
  test-suite holds (``ferminet/tests/hamiltonian_test.py:65-250``,
  ``ferminet/tests/network_blocks_test.py:38-45``), re-expressed in
  ``tests/test_oracle_known_answers.py``.
* The AIQMC network forward itself has NO reference-produced golden vector:
  JAX is not installed in this image, so the reference cannot be run, and the
  committed ``.npz`` checkpoints belong to superseded network versions
  (SURVEY.md F7).  Network-forward parity is therefore "unpinned" against the
  reference; it is cross-checked between two independent restatements
  (``network`` in torch and ``network_np`` in numpy) and by finite differences.
"""
