"""packnet_sfm/utils/misc.py helpers used on the path."""


def filter_dict(dictionary, keywords):
    return [key for key in keywords if key in dictionary]


def make_list(var, n=None):
    var = var if isinstance(var, list) else [var]
    if n is None:
        return var
    assert len(var) == 1 or len(var) == n, "Wrong list length for make_list"
    return var * n if len(var) == 1 else var


def parse_crop_borders(borders, shape):
    """Crop box (left, top, right, bottom) from a crop spec.  utils/misc.py:77-146.

    borders: () -> the full image; (y, height, x, width) -> 4-tuple form; (y, x) -> 2-tuple form.
    Integers crop regularly (negative = counted from the far border; a non-positive height /
    width extends to the border), floats centre the crop at that fraction of the size.
    shape: (image_height, image_width).
    """
    H, W = shape
    if len(borders) == 0:
        return 0, 0, W, H
    if len(borders) == 4:
        y, h, x, w = borders

        def axis(start, extent, size):
            if isinstance(start, int):
                lo = start + size if start < 0 else start
                hi = extent + size if extent <= 0 else extent + lo
                return lo, hi
            center, half = start * size, extent / 2
            return int(center - half), int(center + half)

        left, right = axis(x, w, W)
        top, bottom = axis(y, h, H)
        box = (left, top, right, bottom)
    elif len(borders) == 2:
        y, x = borders
        if isinstance(x, int):
            box = (max(0, x), max(0, y), W + min(0, x), H + min(0, y))
        else:
            cw, half_w = x * W, y / 2
            ch, half_h = x * H, y / 2
            box = (int(cw - half_w), int(ch - half_h), int(cw + half_w), int(ch + half_h))
    else:
        raise NotImplementedError("Crop tuple must have 2 or 4 values.")
    assert 0 <= box[0] < box[2] <= W and 0 <= box[1] < box[3] <= H, \
        "Crop borders {} are invalid".format(box)
    return box
