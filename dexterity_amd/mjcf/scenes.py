"""Scene definitions: what `manipulation.load(...)` assembles in the reference.

Each function mirrors the composition done by a reference task constructor and
returns a compiled model.  They read the vendor MJCF/STL files of the reference
checkout, so they only run at asset-build time (`tools/build_assets.py`); the
compiled blobs under `assets/` are what the runtime (and the GPU box) loads.

* `shadow_reorient`  -- `manipulation/tasks/reorient.py:324-364`: Standard arena
  ground (`models/arenas/standard.py:16-23`), Shadow hand at the palm-upright pose
  (`models/hands/shadow_hand_e.py:13-14`), free OpenAI cube of half-size 0.02
  (`reorient.py:47,134`), dt 0.005.  The hint cube (`reorient.py:138-141`) is a
  contact-free mocap body with no effect on dynamics and is not compiled.
* `adroit_reach`     -- `manipulation/tasks/reach.py:223-249`: Adroit hand, ground
  collisions disabled (`reach.py:131-132`), dt 0.02.
* `shadow_reach`     -- BASELINE.json config 2 naming (reach with the Shadow hand,
  contact-free smooth dynamics), dt 0.02.
* `adroit_hand`      -- the Adroit hand alone (the reference's hands_test.py physics
  known-answer tests), dt 0.002, iterations 20.
* `bimanual_handover` -- BASELINE.json config 5 (synthetic; the reference has no
  bimanual task): two Shadow hands welded to the world palm-up side by side at the
  Juggle task's x offsets (`juggle.py:22-26`, +-0.1 m, here +-0.12 m so the palms do not
  overlap), the reorient cube on the left palm, dt 0.005 as reorient.  nq 55 / nv 54.
"""

from __future__ import annotations

import os

from dexterity_amd.mjcf.compiler import Scene

REFERENCE_ROOT = os.environ.get("DEXTERITY_REFERENCE", "/root/reference")
_VENDOR = os.path.join(REFERENCE_ROOT, "dexterity", "models", "vendor")
SHADOW_XML = os.path.join(
    _VENDOR, "shadow_robot", "shadow_hand_description", "mjcf", "shadow_hand_series_e.xml"
)
ADROIT_XML = os.path.join(_VENDOR, "adroit", "adroit_hand_description", "mjcf", "adroit_hand.xml")

# models/hands/shadow_hand_e.py:13-14 and adroit_hand.py:13-14.
PALM_UPRIGHT_POS = (0.0, 0.2, 0.1)
PALM_UPRIGHT_QUAT = (0.0, 0.0, 0.707106781186, -0.707106781186)
SHADOW_FINGERTIPS = ("fftip", "mftip", "rftip", "lftip", "thtip")  # shadow_hand_e_constants.py:356
ADROIT_FINGERTIP_SITES = ("S_fftip", "S_mftip", "S_rftip", "S_lftip", "S_thtip")

# Cube reorientation spawn box, reorient.py:70-78.
PROP_BBOX_LOWER = (-0.025, -0.155, 0.16)
PROP_BBOX_UPPER = (0.025, -0.105, 0.16)


def _ground(scene: Scene, collide: bool) -> None:
    # models/arenas/standard.py:16-23.
    kw = dict(friction="0.4 0.005 0.0001", solimp="0.95 0.99 0.001", solref="0.002 1")
    if not collide:
        kw.update(contype="0", conaffinity="0")
    scene.add_world_geom("ground", "plane", (1, 1, 0.1), **kw)


def shadow_reorient():
    scene = Scene(timestep=0.005)
    _ground(scene, collide=True)
    scene.attach_mjcf(SHADOW_XML, "shadow_hand_e/", PALM_UPRIGHT_POS, PALM_UPRIGHT_QUAT)
    for tip in SHADOW_FINGERTIPS:
        scene.add_site("shadow_hand_e/" + tip, "shadow_hand_e/" + tip + "_site")
    centre = [(a + b) / 2 for a, b in zip(PROP_BBOX_LOWER, PROP_BBOX_UPPER)]
    scene.add_free_box("prop", 0.02, centre)
    return scene.compile()


def shadow_reach():
    scene = Scene(timestep=0.02)
    _ground(scene, collide=False)
    scene.attach_mjcf(SHADOW_XML, "shadow_hand_e/", PALM_UPRIGHT_POS, PALM_UPRIGHT_QUAT)
    for tip in SHADOW_FINGERTIPS:
        scene.add_site("shadow_hand_e/" + tip, "shadow_hand_e/" + tip + "_site")
    scene.disable_contact = True
    return scene.compile()


def adroit_reach():
    scene = Scene(timestep=0.02)
    _ground(scene, collide=False)
    scene.attach_mjcf(ADROIT_XML, "adroit_hand/", PALM_UPRIGHT_POS, PALM_UPRIGHT_QUAT)
    return scene.compile()


def adroit_hand():
    """The Adroit hand alone, as `mjcf.Physics.from_mjcf_model(AdroitHand().mjcf_model)`
    builds it in the reference's hand tests (hands_test.py:167-169, 211-212): the
    vendor MJCF is the root model, so its own `<option iterations="20">`
    (adroit_hand.xml:12) applies and the timestep is MuJoCo's default 0.002 s; no
    arena, no ground, the hand at its MJCF pose."""
    scene = Scene(timestep=0.002)
    scene.iterations = 20
    scene.attach_mjcf(ADROIT_XML, "adroit_hand/")
    return scene.compile()


BIMANUAL_OFFSET = 0.12


def bimanual_handover():
    scene = Scene(timestep=0.005)
    _ground(scene, collide=True)
    for side, dx in (("left", BIMANUAL_OFFSET), ("right", -BIMANUAL_OFFSET)):
        prefix = f"shadow_hand_{side}/"
        pos = (PALM_UPRIGHT_POS[0] + dx, PALM_UPRIGHT_POS[1], PALM_UPRIGHT_POS[2])
        scene.attach_mjcf(SHADOW_XML, prefix, pos, PALM_UPRIGHT_QUAT)
        for tip in SHADOW_FINGERTIPS:
            scene.add_site(prefix + tip, prefix + tip + "_site")
    centre = [(a + b) / 2 for a, b in zip(PROP_BBOX_LOWER, PROP_BBOX_UPPER)]
    centre[0] += BIMANUAL_OFFSET
    scene.add_free_box("prop", 0.02, centre)
    return scene.compile()


SCENES = {
    "shadow_reorient": shadow_reorient,
    "shadow_reach": shadow_reach,
    "adroit_reach": adroit_reach,
    "adroit_hand": adroit_hand,
    "bimanual_handover": bimanual_handover,
}
