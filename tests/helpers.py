"""Shared assertions for parity tests (GPU path vs CPU oracle)."""
import numpy as np

FIELDS = ("flag", "pos", "score", "n_cigar", "hits")


def assert_records_equal(gpu: dict, ref: dict, reads=None, max_show=5):
    """Bit-exact equality of every per-read field; CIGAR compared on its first n_cigar ops."""
    bad = np.zeros(len(ref["flag"]), dtype=bool)
    for k in FIELDS:
        bad |= np.asarray(gpu[k]) != np.asarray(ref[k])
    nc = np.asarray(ref["n_cigar"])
    cg, cr = np.asarray(gpu["cigar"]), np.asarray(ref["cigar"])
    col = np.arange(cr.shape[1])[None, :]
    live = col < nc[:, None]
    bad |= ((cg != cr) & live).any(axis=1)
    idx = np.nonzero(bad)[0]
    if len(idx):
        lines = []
        for r in idx[:max_show]:
            lines.append(f"read {r}: " + " ".join(f"{k}={int(gpu[k][r])}/{int(ref[k][r])}" for k in FIELDS)
                         + f" cigar={list(cg[r][:nc[r]])}/{list(cr[r][:nc[r]])}"
                         + (f" seq={bytes(reads[r]).decode()}" if reads is not None else ""))
        raise AssertionError(f"{len(idx)} of {len(bad)} reads differ (gpu/oracle):\n" + "\n".join(lines))
