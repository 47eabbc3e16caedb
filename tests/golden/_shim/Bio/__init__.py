"""Stub so the reference's read_data module imports; MAF parsing via Biopython is unavailable."""
