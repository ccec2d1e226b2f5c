"""Camera calibrations of the reference's example settings (K = fx fy cx cy,
D = OpenCV k1 k2 p1 p2 [k3] [k4 k5 k6]); Tracking.cc:165-199 reads them as float."""
EUROC = ((458.654, 457.296, 367.215, 248.375),            # Examples/Monocular/EuRoC.yaml:8-16
         (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05), (752, 480))
TUM1 = ((517.306408, 516.469215, 318.643040, 255.313989),  # Examples/Monocular/TUM1.yaml:8-17
        (0.262383, -0.953104, -0.005358, 0.002628, 1.163314), (640, 480))
# synthetic rational (bUseDistK6, Tracking.cc:190-199) model: k1 k2 p1 p2 k3 k4 k5 k6
RATIONAL = ((400.0, 401.5, 330.25, 241.75),
            (0.12, -0.05, 0.0011, -0.0007, 0.004, 0.31, -0.02, 0.005), (640, 480))
# odd size (no 4-pixel vector path), off-centre principal point
ODD = ((300.0, 310.0, 150.5, 90.25), (-0.2, 0.05, 0.001, -0.002), (301, 183))
# strong pincushion, short focal length: corner tiles read source boxes too
# large for LDS (the global-gather path) or entirely outside the image
WILD = ((150.0, 150.0, 320.0, 240.0), (0.9, 0.1, 0.0, 0.0), (640, 480))
ALL = {"wild": WILD, "euroc": EUROC, "tum1": TUM1, "rational": RATIONAL, "odd": ODD}
