"""Inner Anderson acceleration (reference lib/AndersonAcceleration.py).

Active when ``inner accel order > 0`` (reference lib/Preconditioner.py:248-249):
libpls.so mixes consecutive PC outputs on the device inside the block-PC apply
(option ``pls.inner_accel_order``).  This class records the order for API
parity; the mixing itself is not callable from Python.
"""


class AndersonAcceleration:
    def __init__(self, order):
        self.order = order
        self.k = 0

    def get_next_vector(self, gk):
        raise NotImplementedError("inner Anderson mixing runs inside libpls.so's PC apply "
                                  "(set 'inner accel order' in the parameters)")
