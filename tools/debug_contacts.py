"""Per-contact GPU vs oracle dump for the parity states (development aid)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dexterity_amd import _lib, physics
from dexterity_amd.mjcf.compiler import CompiledModel
from tests.test_gpu_parity import _oracle_states, _oracle_forward, _load_states
from oracle import oracle as O
O.build()
cm = CompiledModel.load("assets/shadow_reorient.npz")
xfrc = physics.gravity_compensation(cm, "shadow_hand_e/")
om, states = _oracle_states(O, cm, xfrc)
model = physics.Model(cm)
phys = _load_states(physics, model, xfrc, states)
phys.debug(True); phys.forward(); phys.sync()
con = phys.debug_get("contact"); qacc = phys.qacc
for e, st in enumerate(states):
    d = _oracle_forward(O, om, cm, xfrc, st)
    oc = {(int(r[13]), int(r[14])): r for r in d.contacts()}
    gc = con[e, : (con[e, :, 15] != 0).sum()]
    print(f"env {e}: ncon gpu {len(gc)} oracle {len(oc)}  qacc err {np.abs(qacc[e]-d.qacc).max():.2e}")
    for r in gc:
        o = oc.get((int(r[13]), int(r[14])))
        if o is None: print("   extra gpu contact", r[13:15]); continue
        dp = np.abs(r[0:3]-o[0:3]).max(); dn = np.abs(r[3:6]-o[3:6]).max()
        flag = " <<<" if dp > 1e-4 or dn > 1e-3 else ""
        print(f"   pair {int(r[13])},{int(r[14])} dist g {r[12]:.3e} o {o[12]:.3e} dpos {dp:.2e} dn {dn:.2e}{flag}")
        if flag: print("      gpu pos", r[0:3], "n", r[3:6], "\n      orc pos", o[0:3], "n", o[3:6])
