"""Month-end calendar arithmetic on integer month indices.

The reference does all date logic with pandas offsets (``MonthEnd``, ``relativedelta``,
``date_range(freq='MS') - 1 day``).  The engine keys every monthly panel by an integer
month index ``mi = 12*year + (month-1)`` so that lags, windows and joins are integer ops
that can live on the device.  Helpers here convert both ways and reproduce the reference's
date grids (PFML_Input_Data.py:133-154).
"""
from __future__ import annotations

import numpy as np
import pandas as pd


_EPOCH_MI = 1970 * 12                  # month index of numpy's datetime64[M] zero


def month_index(dates) -> np.ndarray:
    """Timestamp(s) -> integer month index (12*year + month-1).  Naive datetime64 arrays take
    a pure numpy path (datetime64[M] arithmetic); anything else goes through pandas."""
    a = np.atleast_1d(np.asarray(dates))
    if np.issubdtype(a.dtype, np.datetime64) and not np.isnat(a).any():
        if a.size > 4096:
            # panels repeat few distinct dates: convert the distinct values only (the
            # datetime64[M] cast is calendar arithmetic per element)
            codes, uniq = pd.factorize(a.view(np.int64), sort=False)
            return (uniq.view(a.dtype).astype("datetime64[M]").astype(np.int64) + _EPOCH_MI)[codes]
        return a.astype("datetime64[M]").astype(np.int64) + _EPOCH_MI
    d = pd.DatetimeIndex(pd.to_datetime(np.atleast_1d(dates)))
    return (d.year.to_numpy().astype(np.int64) * 12 + d.month.to_numpy().astype(np.int64) - 1)


def month_end(mi) -> pd.DatetimeIndex:
    """Integer month index -> month-end Timestamp(s) (first day of the next month - 1 day)."""
    mi = np.atleast_1d(np.asarray(mi, dtype=np.int64))
    if mi.size > 4096:                  # few distinct months: convert those, then take
        codes, uniq = pd.factorize(mi, sort=False)
        return month_end(uniq)[codes]
    nxt = (mi - _EPOCH_MI + 1).astype("datetime64[M]").astype("datetime64[D]")
    return pd.DatetimeIndex((nxt - np.timedelta64(1, "D")).astype("datetime64[ns]"))


def eom(ts) -> pd.Timestamp:
    return pd.Timestamp(ts) + pd.offsets.MonthEnd(0)


def monthly_grid(start_mi: int, end_mi: int) -> np.ndarray:
    """Inclusive range of month indices."""
    return np.arange(int(start_mi), int(end_mi) + 1, dtype=np.int64)


def pfml_date_grids(first_cov_mi: int, lb_hor: int, test_end: pd.Timestamp,
                    start_year: int, split_years: int) -> dict:
    """Month grids used by the PFML stages.

    * ``m2``  - months with PFML inputs: first covariance month + lb_hor + 1 .. the month
      before ``test_end`` (PFML_Input_Data.py:136-140).
    * ``oos`` - out-of-sample months, Dec of (start_year+split_years-1) .. month before
      test_end (PFML_Input_Data.py:142-146: ``date_range(start_oos-01-01, ..., 'MS') - 1d``).
    * ``lb``  - months for which vol scales are needed (m2 widened by lb_hor+1 months back).
    """
    last = int(month_index(test_end)[0]) - 1
    start_m2 = first_cov_mi + lb_hor + 1
    start_oos = (start_year + split_years) * 12 + 0 - 1   # Jan of start_oos minus one month
    return {
        "m2": monthly_grid(start_m2, last),
        "oos": monthly_grid(start_oos, last),
        "lb": monthly_grid(start_m2 - (lb_hor + 1), last),
    }


def year_of(mi) -> np.ndarray:
    return np.asarray(mi, dtype=np.int64) // 12


def month_of(mi) -> np.ndarray:
    return np.asarray(mi, dtype=np.int64) % 12 + 1


def mi_from_ym(year: int, month: int) -> int:
    return int(year) * 12 + int(month) - 1
