"""ARTIC-style primer scheme parsing — same results as the reference's ``load_scheme``
(/root/reference/basecount/scheme.py:3-78, itself from swell by Sam Nicholls).

For every primer line ``<chrom> <start> <end> <scheme>_<tile>_<side...>``:
  * a LEFT primer widens the tile's outer start to the leftmost primer start and its inner
    start to the rightmost LEFT primer end (scheme.py:19-29);
  * a RIGHT primer widens the outer end to the rightmost end and the inner end to the leftmost
    RIGHT primer start (scheme.py:31-41);
tiles with both an inner start and an inner end are kept once, in first-appearance order,
then sorted by integer tile number (scheme.py:43-59); with ``clip`` each inner window is
clipped to the previous tile's outer end and the next tile's outer start (scheme.py:60-74).
Returns ``[(scheme, tile, {"start", "inside_start", "inside_end", "end"}), ...]``.
"""
from __future__ import annotations


def _records(fh, ints):
    for line in fh:
        data = line.strip().split()
        if ints:  # the first pass converts the coordinates before splitting the name
            coords = (int(data[1]), int(data[2]))
        else:
            coords = (data[1], data[2])
        scheme, tile, side = data[3].split("_", 2)
        yield coords, scheme, tile, side


def load_scheme(bed, clip=True):
    windows: dict = {}
    with open(bed) as fh:
        for (start, end), _scheme, tile, side in _records(fh, True):
            w = windows.setdefault(tile, {"start": -1, "inside_start": -1, "inside_end": -1,
                                          "end": -1})
            up = side.upper()
            if "LEFT" in up:
                if w["start"] == -1:
                    w["start"], w["inside_start"] = start, end
                w["start"] = min(w["start"], start)
                w["inside_start"] = max(w["inside_start"], end)
            elif "RIGHT" in up:
                if w["end"] == -1:
                    w["end"], w["inside_end"] = end, start
                w["end"] = max(w["end"], end)
                w["inside_end"] = min(w["inside_end"], start)

        fh.seek(0)
        tiles, seen = [], set()
        for _coords, scheme, tile, _side in _records(fh, False):
            w = windows[tile]
            if w["inside_start"] != -1 and w["inside_end"] != -1 and tile not in seen:
                tiles.append((scheme, tile, w))
                seen.add(tile)

        tiles = sorted(tiles, key=lambda x: int(x[1]))
        if not clip:
            return tiles
        out = []
        for i, (scheme, tile, w) in enumerate(tiles):
            d = dict(w)
            if i > 0:
                d["inside_start"] = tiles[i - 1][2]["end"]
            if i < len(tiles) - 1:
                d["inside_end"] = tiles[i + 1][2]["start"]
            out.append((scheme, tile, d))
        return out
