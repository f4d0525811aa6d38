"""aiqmc -- MI355X-native drop-in for the AIQMCrelease3 VMC hot path.

Module paths mirror the reference package (AIQMCrelease3):
  aiqmc.wavefunction_Ynlm.nn       make_ai_net, AINetData, Network
  aiqmc.Energy.hamiltonian         local_energy, potential_*
  aiqmc.VMC.VMCmcstep              main_monte_carlo, walkers_update, limdrift
  aiqmc.constants                  pmean / psum / all_gather over torch.distributed (RCCL)
  aiqmc.spin_indices               jastrow_indices_ee, spin_indices_h
  aiqmc.initial_electrons_positions.init   init_electrons
  aiqmc.utils.utils                select_output
Compute runs in hand-written HIP kernels for gfx950 (libaiqmc_hip.so, C-ABI in
include/aiqmc.h); there is no CPU fallback.
"""
__version__ = "0.1.0"
