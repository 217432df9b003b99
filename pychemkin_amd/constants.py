"""cgs constants, same values as the reference (``constants.py:26-38``).

With ``R_GAS = BOLTZMANN * AVOGADRO`` and the Chemkin atomic weights these reproduce the
``simple.baseline`` air density to 2e-16.
"""

BOLTZMANN = 1.3806504e-16  # [erg/K]
AVOGADRO = 6.02214179e23  # [1/mol]
P_ATM = 1.01325e06  # [dyn/cm2]
P_TORRS = P_ATM / 760.0
ERGS_PER_JOULE = 1.0e7
JOULES_PER_CALORIE = 4.184e0
ERGS_PER_CALORIE = JOULES_PER_CALORIE * ERGS_PER_JOULE
ERGS_PER_EV = 1.602176487e-12
EV_PER_K = ERGS_PER_EV / BOLTZMANN
R_GAS = BOLTZMANN * AVOGADRO  # [erg/mol-K]
R_GAS_CAL = R_GAS * 1.0e-7 / JOULES_PER_CALORIE  # [cal/mol-K]


class Air:
    """Air recipe, upper-case symbols (reference ``constants.py:42-55``)."""

    @staticmethod
    def X():
        return [("O2", 0.21), ("N2", 0.79)]

    @staticmethod
    def Y():
        return [("O2", 0.23), ("N2", 0.77)]


class air:
    """Air recipe, lower-case symbols (reference ``constants.py:58-71``)."""

    @staticmethod
    def X():
        return [("o2", 0.21), ("n2", 0.79)]

    @staticmethod
    def Y():
        return [("o2", 0.23), ("n2", 0.77)]
