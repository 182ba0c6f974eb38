"""Camera intrinsic calibration from checkerboard views (no OpenCV in this environment).

Capabilities of ``/root/reference/scripts/01_calibrate_camera.py:21-123``: checkerboard (9, 7)
inner corners with 0.027 m squares, corner detection + sub-pixel refinement (11x11 window,
30 iterations / 0.001 eps), at least 5 captures, ``calibrateCamera`` -> ``mtx, dist, rvecs, tvecs``
saved to an npz, mean reprojection error report. Implemented as:

  * :mod:`.board`    -- object points and a synthetic board renderer (pinhole + Brown distortion)
  * :mod:`.corners`  -- saddle-point corner detector, grid ordering, ``corner_subpix``
  * :mod:`.zhang`    -- Zhang's closed form + Levenberg-Marquardt refinement of
                        (fx, fy, cx, cy, k1, k2, p1, p2, k3) and per-view poses; ``project_points``
"""
from .board import object_points, render_board_view, random_board_pose
from .corners import corner_subpix, find_chessboard_corners
from .zhang import calibrate_camera, project_points, reprojection_errors, rodrigues

__all__ = ["object_points", "render_board_view", "random_board_pose", "find_chessboard_corners", "corner_subpix",
           "calibrate_camera", "project_points", "reprojection_errors", "rodrigues"]
