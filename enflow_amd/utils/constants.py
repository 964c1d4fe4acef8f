"""Physical constants in the reference's LJ unit system (enflow/utils/constants.py:1-7).

The reference reads the argon atomic weight from rdkit's periodic table; rdkit
is not part of this framework, so the value it returns (39.948 amu) is fixed
here.
"""
M = 39.948          # amu, argon (rdkit GetAtomicWeight('Ar'))
sigma = 3.4e-10     # m
eps = 0.238e3       # J/mol
kB = 8.3144621      # J/(K mol)

atom_types = {'H': 0, 'C': 1, 'N': 2, 'O': 3, 'F': 4}
