"""Per-contact and per-state GPU-vs-oracle differences over a wide sample of reorient
states (the states of tests/test_gpu_parity.py's wide-sample test): for each contact
the depth, depth error, point displacement (along / across the normal) and normal
angle; for each state the hand-dof and cube-dof qacc errors relative to the forcing
scale.  Prints one line per contact and per state.

  python tools/parity_survey.py [n_traj] [seed]
"""

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dexterity_amd import build, physics  # noqa: E402
from dexterity_amd.mjcf.compiler import CompiledModel  # noqa: E402
from tests.conftest import ROOT  # noqa: E402
from tests.test_gpu_parity import _load_states, _oracle_forward, _oracle_states, _separation  # noqa: E402


def main():
    n_traj = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    build.build()
    from oracle import oracle as oracle_mod

    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    xfrc = physics.gravity_compensation(cm, "shadow_hand_e/")
    om, states = _oracle_states(oracle_mod, cm, xfrc, n_traj=n_traj, seed=seed)
    model = physics.Model(cm)
    ph = _load_states(physics, model, xfrc, states)
    ph.debug(True)
    ph.forward()
    ph.sync()
    con = ph.debug_get("contact")
    qacc = ph.qacc
    for e, st in enumerate(states):
        d = _oracle_forward(oracle_mod, om, cm, xfrc, st)
        oc = {(int(r[13]), int(r[14])): r for r in d.contacts()}
        worst = 0.0
        for r in con[e, : (con[e, :, 15] != 0).sum()]:
            key = (int(r[13]), int(r[14]))
            o = oc.get(key)
            if o is None:
                print(f"state {e} contact {key} missing in oracle")
                continue
            delta = r[0:3] - o[0:3]
            along = float(np.dot(delta, o[3:6]))
            ang = float(np.linalg.norm(r[3:6] - o[3:6]))
            worst = max(worst, ang)
            sg = _separation(cm, d, key[0], key[1], r[3:6]) - o[12]
            so = _separation(cm, d, key[0], key[1], o[3:6]) - o[12]
            print(f"state {e} pair {key} dist {o[12]:+.3e} ddist {r[12] - o[12]:+.1e} "
                  f"dpos {np.abs(delta).max():.1e} along {along:+.1e} normal {ang:.1e} "
                  f"normal*dist {ang * abs(o[12]):.1e} sep_gpu {sg:+.1e} sep_oracle {so:+.1e}")
        scale = max(1.0, np.abs(d.qacc_smooth).max())
        err = np.abs(qacc[e] - d.qacc)
        print(f"STATE {e} ncon {len(oc)} scale {scale:.2f} hand {err[:cm.nv - 6].max() / scale:.1e} "
              f"cube {err[cm.nv - 6:].max() / scale:.1e} worst_normal {worst:.1e}")
    ph.close()


if __name__ == "__main__":
    main()
