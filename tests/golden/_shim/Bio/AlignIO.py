def parse(*a, **k):
    raise RuntimeError("Biopython is not installed in this container")
