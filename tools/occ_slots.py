"""Prints the substep queue's persistent workgroups (resident step-kernel workgroups per
CU x CUs) of a reorient batch; DX_LDS_PAD adds (or, negative, removes) LDS bytes per
workgroup in that count.  Creates the batch only: nothing is launched."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dexterity_amd.physics import BatchedPhysics, Model  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
m = Model.from_file(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
b = BatchedPhysics(m, 64, 0)
s = b.debug_get("queue_slots")
print("lds", m.lds_bytes, "pad", os.environ.get("DX_LDS_PAD", "0"), "slots", int(s[0]), flush=True)
