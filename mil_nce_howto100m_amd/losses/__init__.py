"""Loss registry: MIL-NCE (the trained objective) and the soft-DTW alignment family."""
from .milnce import MILNCELoss


def build_loss(args):
    name = getattr(args, "loss", "milnce")
    if name == "milnce":
        return MILNCELoss()
    from . import sdtw
    table = {"cdtw": sdtw.CDTW, "sdtw_cidm": sdtw.SDTW_CIDM, "sdtw_negative": sdtw.SDTW_negative,
             "sdtw_3": sdtw.SDTW_3}
    if name not in table:
        raise ValueError(f"unknown loss {name}")
    return table[name](args)


__all__ = ["MILNCELoss", "build_loss"]
