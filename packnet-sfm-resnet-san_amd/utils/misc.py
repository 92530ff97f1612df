"""packnet_sfm/utils/misc.py helpers used on the path."""


def filter_dict(dictionary, keywords):
    return [key for key in keywords if key in dictionary]


def make_list(var, n=None):
    var = var if isinstance(var, list) else [var]
    if n is None:
        return var
    assert len(var) == 1 or len(var) == n, "Wrong list length for make_list"
    return var * n if len(var) == 1 else var
