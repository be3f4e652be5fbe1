"""Host-side camera and GUI parameters, mirrored from the reference.

* :class:`Camera`          <- Utils/camera.h:8-75 (orbit camera; any move resets frameCounter, :71)
* :class:`parameter_config` <- Utils/gui_config.h:19-46 (the ImGui slider defaults)
* glm helpers (perspective / lookAt / rigid inverse) in float32, column-major
  16-float arrays in ``glm::value_ptr`` order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

f32 = np.float32


def radians(deg: float) -> np.float32:
    return f32(deg) * f32(0.01745329251994329576923690768489)


def perspective(fovy: np.float32, aspect: np.float32, znear: np.float32, zfar: np.float32) -> np.ndarray:
    """glm::perspective (RH, depth -1..1)."""
    t = f32(math.tan(float(f32(fovy) / f32(2))))
    m = np.zeros(16, np.float32)
    m[0] = f32(1) / (f32(aspect) * t)
    m[5] = f32(1) / t
    m[10] = -(f32(zfar) + f32(znear)) / (f32(zfar) - f32(znear))
    m[11] = f32(-1)
    m[14] = -(f32(2) * f32(zfar) * f32(znear)) / (f32(zfar) - f32(znear))
    return m


def _normalize(v: np.ndarray) -> np.ndarray:
    v = v.astype(np.float32)
    d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]
    return v * (f32(1) / f32(np.sqrt(d)))


def _cross(a, b):
    return np.array([a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]], np.float32)


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def look_at(eye, center, up) -> np.ndarray:
    """glm::lookAt (RH)."""
    eye = np.asarray(eye, np.float32)
    f = _normalize(np.asarray(center, np.float32) - eye)
    s = _normalize(_cross(f, np.asarray(up, np.float32)))
    u = _cross(s, f)
    m = np.eye(4, dtype=np.float32).reshape(16)  # column-major: m[c*4+r]
    m[0], m[4], m[8] = s
    m[1], m[5], m[9] = u
    m[2], m[6], m[10] = -f
    m[12] = -_dot(s, eye)
    m[13] = -_dot(u, eye)
    m[14] = _dot(f, eye)
    return m


def rigid_inverse(view: np.ndarray) -> np.ndarray:
    """inverse(view) for a rotation+translation view matrix (main.cpp:445)."""
    v = np.asarray(view, np.float32).reshape(16)
    r = np.zeros(16, np.float32)
    for row in range(3):
        for col in range(3):
            r[col * 4 + row] = v[row * 4 + col]
    t = v[12:15]
    for row in range(3):
        r[12 + row] = -((r[row] * t[0] + r[4 + row] * t[1]) + r[8 + row] * t[2])
    r[15] = f32(1)
    return r


def mat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """glm mat4*mat4 (column-major; Result[i] = A0*B[i][0] + A1*B[i][1] + A2*B[i][2] + A3*B[i][3])."""
    a = np.asarray(a, np.float32).reshape(16)
    b = np.asarray(b, np.float32).reshape(16)
    o = np.zeros(16, np.float32)
    for c in range(4):
        for r in range(4):
            o[c * 4 + r] = ((a[r] * b[c * 4] + a[4 + r] * b[c * 4 + 1]) + a[8 + r] * b[c * 4 + 2]) + a[12 + r] * b[c * 4 + 3]
    return o


class Camera:
    """Utils/camera.h:8-75, headless: `orbit()` replaces the mouse callbacks (main.cpp:614-655)."""

    def __init__(self, width: int = 800, height: int = 800):
        self.width = int(width)
        self.height = int(height)
        self.near_plane = f32(0.01)
        self.far_plane = f32(1000.0)
        self.fov_y = f32(90.0)
        self.upAngle = f32(10.0)
        self.rotatAngle = f32(0.0)
        self.r_dis = f32(2.0)
        self.move_vec = np.zeros(3, np.float32)
        self.look_at_point = np.zeros(3, np.float32)
        self.frameCounter = 0
        self.dirty = False
        self.cam_position = self._orbit_eye()
        self.cam_proj_mat = perspective(radians(90.0), f32(self.width) / f32(self.height), self.near_plane,
                                        self.far_plane)
        self.cam_view_mat = look_at(self.cam_position, self.move_vec, [0, 1, 0])

    def _orbit_eye(self) -> np.ndarray:
        ra, ua = float(radians(float(self.rotatAngle))), float(radians(float(self.upAngle)))
        e = np.array([-math.sin(ra) * math.cos(ua), math.sin(ua), math.cos(ra) * math.cos(ua)], np.float32)
        return e * self.r_dis

    def orbit(self, d_rot_deg: float = 0.0, d_up_deg: float = 0.0) -> None:
        """cursor_position_callback (main.cpp:614-630): resets frameCounter, marks dirty."""
        self.frameCounter = 0
        self.rotatAngle = f32(self.rotatAngle + f32(d_rot_deg))
        self.upAngle = f32(min(max(float(self.upAngle + f32(d_up_deg)), -89.0), 89.0))
        self.dirty = True

    def update(self) -> None:
        """Camera::update (camera.h:62-74)."""
        if self.dirty:
            eye = self._orbit_eye() + self.move_vec
            self.cam_position = eye.astype(np.float32)
            self.look_at_point = self.move_vec.copy()
            self.cam_view_mat = look_at(self.cam_position, self.look_at_point, [0, 1, 0])
            self.frameCounter = 0
            self.dirty = False


@dataclass
class parameter_config:
    """Utils/gui_config.h:19-46 defaults; accumulate_color defaults False for 1spp+SVGF runs."""

    sigma_z: float = 1.0
    sigma_n: float = 128.0
    sigma_l: float = 4.0
    reproj_normal_threshold: float = 16.0
    reproj_depth_threshold: float = 10.0
    clamp_threshold: float = 10.0
    max_tracing_depth: int = 2
    num_atrous_iterations: int = 5
    accumulate_color: bool = False
    use_normal_texture: bool = False
