"""CPU oracle of the reference rasterizer -- test infrastructure only (see oracle.py)."""
