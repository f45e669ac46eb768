"""Camera poses as ``Input`` scripts.

Each tuple is (up, down, left, right, mouse.x, mouse.y) -- one ``updateAndRender`` call
(``render-cpp/render.hpp:15-21``).  Every script is preceded by one all-zero call (the first call
initialises the scene and forces a camera-matrix update, ``render.cpp:266-270``).  Timed frames
repeat the last tuple with the movement keys zeroed, so the camera holds still
(``render.cpp:136-150``: no key > 0 and an unchanged mouse leave the pose as it is).
"""
from __future__ import annotations

POSES = {
    # identity camera: floor + textured triangle in view
    'P_id': [],
    # elevated overview of every object
    'P_over': [(0, 0, 0, 0, 0, -150), (0, 150, 0, 0, 0, -150), (0, 0, 0, 0, 0, -90)],
    # tetrahedra fill the view (colour path)
    'P_tetra': [(0, 0, 0, 0, -333, 120), (80, 0, 0, 0, -333, 120)],
    # camera at z = -6, inside the floor span: the floor is near-plane clipped
    'P_clip': [(60, 0, 0, 0, 0, 0)],
    # strafe + yaw: exercises translation with the pre-rotation axes (render.cpp:136-139)
    'P_strafe': [(0, 0, 0, 30, 40, 0), (5, 0, 12, 0, 90, -20)],
    # walked forward over the floor: floor-dominated frame, texture magnification + clipping
    'P_floor': [(0, 0, 0, 0, 0, -50), (30, 0, 0, 0, 0, -50)],
}


def script(name: str):
    """The full call sequence for a pose: the zero call, the pose tuples."""
    return [(0, 0, 0, 0, 0, 0)] + list(POSES[name])


def hold(name: str):
    """The tuple timed frames repeat (last mouse position, no movement keys)."""
    s = script(name)
    last = s[-1]
    return (0, 0, 0, 0, last[4], last[5])
