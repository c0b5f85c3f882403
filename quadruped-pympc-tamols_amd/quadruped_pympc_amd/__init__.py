"""MI355X-native sampling SRBD MPC + TAMOLS foothold search behind the Quadruped-PyMPC plugin API.

Host-side mirror of the reference's controller interface; all compute runs in
``libsrbd_hip.so`` (hand-written CDNA4 kernels, C-ABI in ``include/srbd_mpc.h``).
"""
__version__ = "0.1.0"
