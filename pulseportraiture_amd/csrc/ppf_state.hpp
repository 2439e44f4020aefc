// ppf_state.hpp -- per-sub-integration solver state shared by the solver
// (ppf_solve.hip) and the fused moment kernel (ppf_xspec.hip).
#pragma once
#include "ppf_device.hpp"

namespace ppf {

// ===========================================================================
// per-sub-integration solver state (workspace)
// ===========================================================================
// PH_RESTART: the Newton solver's switch from the channel subset to every
// channel: the pending evaluation is at the accepted point x (not a proposal)
enum { PH_INIT = 0, PH_PROPOSAL = 1, PH_DONE = 2, PH_RESTART = 3 };

struct TRState {
    double x[5];          // accepted point
    double th[5];         // point the next pass evaluates
    double f, g[5], H[15];  // model at x (H upper triangle, all 5 params)
    double radius, pred;
    double nu_fit[3], nu_mean, Sd, dof, phi_guess;
    int k, status, nfev, phase;
    int slot_cur, slot_eval, flagmask, nchanx;
    int scat, hb, g_sum, g_tau;
    int g_alpha, newton, sub, mom16;   // newton: Newton trust region; sub: channel-group stride of
                                       // its warm start (1: every channel; tr_update_newton);
                                       // mom16: 16 band-centred moments (k_moments, PPF_OPT_MOM_X)
    // moment mode (no scattering): two moment sets centred at mc[q]
    int mmode, need_mom, mtarget, macc;
    int mvalid[2], meval, nmom;
    double mc[2][3];
    // box bounds of method='TNC' (pptoas.py:503-513, pptoaslib.py:1041-1053);
    // bnd = 0: none on any fitted parameter (lo = -inf, hi = +inf)
    double lo[5], hi[5];
    int bnd, step_cmd;    // step_cmd: k_tr_step_l's update asked for another pass
    double pnorm;         // Newton solver: |scaled step| of the pending proposal
    int nsubev, sub0;     // evaluations on the channel subset; its initial stride
};

__device__ __forceinline__ int uidx(int i, int j) {     // upper-tri index, i <= j
    return i * 5 - (i * (i - 1)) / 2 + (j - i);
}

}  // namespace ppf
