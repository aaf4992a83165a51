// mc_cal.h -- numpy's calendar datetime64 conversions (the casts between
// year / month units and the linear units), restated from numpy's
// datetime.c: convert_datetime_to_datetimestruct -> (year, month, day) ->
// convert_datetimestruct_to_datetime, with its days_to_yearsdays /
// set_datetimestruct_days / get_datetimestruct_days arithmetic on the
// proleptic Gregorian calendar (int64, wrap-around products, C division where
// numpy uses it, floor division where numpy's extract_unit does).  The time
// of day never survives these casts (a year / month source has none; a year /
// month destination drops it), so the date is carried as a day count.
// tests/test_x80.py::test_calendar_* compare every function with numpy's
// astype on the host (tests/native/host_check.hip).
#pragma once

#include "mc_common.h"

enum McDtUnit { MC_DU_Y = 0, MC_DU_M, MC_DU_W, MC_DU_D, MC_DU_h, MC_DU_m, MC_DU_s, MC_DU_ms, MC_DU_us, MC_DU_ns,
                MC_DU_ps, MC_DU_fs, MC_DU_as };

constexpr int64_t MC_NAT = INT64_MIN;

// numpy's extract_unit_64: floor quotient, *d = the non-negative remainder
MC_HD int64_t mc_cal_extract(int64_t *d, int64_t unit) {
  int64_t div = *d / unit, mod = *d % unit;
  if (mod < 0) {
    mod += unit;
    div -= 1;
  }
  *d = mod;
  return div;
}

MC_HD bool mc_cal_leap(int64_t y) { return (y & 0x3) == 0 && ((y % 100) != 0 || (y % 400) == 0); }

MC_HD int mc_cal_month_len(bool leap, int m) {  // m = 0..11
  constexpr int len[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return len[m] + (leap && m == 1 ? 1 : 0);
}

// days since 1970-01-01 of year / month (1..12) / day (1..31)
MC_HD int64_t mc_cal_days_from_ymd(int64_t year, int month, int64_t day) {
  int64_t y = year - 1970;
  int64_t days = y * 365;
  if (days >= 0) {
    y += 1;          // 1968 is the closest leap year before 1970; exclude the current year
    days += y / 4;
    y += 68;         // 1900: the closest previous year divisible by 100
    days -= y / 100;
    y += 300;        // 1600: divisible by 400
    days += y / 400;
  } else {
    y -= 2;          // 1972 is the closest later leap year; include the current year
    days += y / 4;
    y -= 28;         // 2000: the closest later year divisible by 100 (and by 400)
    days -= y / 100;
    days += y / 400;
  }
  const bool leap = mc_cal_leap(year);
  for (int i = 0; i < month - 1; ++i) days += mc_cal_month_len(leap, i);
  return days + day - 1;
}

// days since 1970-01-01 -> year, month (1..12), day (1..31)
MC_HD void mc_cal_ymd_from_days(int64_t days_in, int64_t *year_out, int *month_out, int64_t *day_out) {
  constexpr int64_t per400 = 400 * 365 + 100 - 4 + 1;
  int64_t days = days_in - (365 * 30 + 7);  // relative to 2000-01-01
  int64_t year;
  if (days >= 0) {
    year = 400 * (days / per400);
    days = days % per400;
  } else {
    year = 400 * ((days - (per400 - 1)) / per400);
    days = days % per400;
    if (days < 0) days += per400;
  }
  if (days >= 366) {
    year += 100 * ((days - 1) / (100 * 365 + 25 - 1));
    days = (days - 1) % (100 * 365 + 25 - 1);
    if (days >= 365) {
      year += 4 * ((days + 1) / (4 * 365 + 1));
      days = (days + 1) % (4 * 365 + 1);
      if (days >= 366) {
        year += (days - 1) / 365;
        days = (days - 1) % 365;
      }
    }
  }
  year += 2000;
  const bool leap = mc_cal_leap(year);
  int month = 12;
  for (int i = 0; i < 12; ++i) {
    const int len = mc_cal_month_len(leap, i);
    if (days < len) {
      month = i + 1;
      break;
    }
    days -= len;
  }
  *year_out = year;
  *month_out = month;
  *day_out = days + 1;
}

MC_HD int64_t mc_cal_wrap_mul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

// one datetime64 value: ticks of (src_unit, src_num) -> ticks of
// (dst_unit, dst_num) through the calendar date
MC_HD int64_t mc_cal_convert(int64_t v, int su, int64_t sn, int du, int64_t dn) {
  if (v == MC_NAT) return MC_NAT;
  int64_t dt = mc_cal_wrap_mul(v, sn);
  int64_t year = 1970, day = 1, days = 0;
  int month = 1;
  bool have_days = false;
  switch (su) {
    case MC_DU_Y: year = 1970 + dt; break;
    case MC_DU_M: year = 1970 + mc_cal_extract(&dt, 12); month = (int)dt + 1; break;
    case MC_DU_W: days = mc_cal_wrap_mul(dt, 7); have_days = true; break;
    case MC_DU_D: days = dt; have_days = true; break;
    case MC_DU_h: days = mc_cal_extract(&dt, 24); have_days = true; break;
    case MC_DU_m: days = mc_cal_extract(&dt, 60LL * 24); have_days = true; break;
    case MC_DU_s: days = mc_cal_extract(&dt, 60LL * 60 * 24); have_days = true; break;
    case MC_DU_ms: days = mc_cal_extract(&dt, 1000LL * 60 * 60 * 24); have_days = true; break;
    case MC_DU_us: days = mc_cal_extract(&dt, 1000LL * 1000 * 60 * 60 * 24); have_days = true; break;
    case MC_DU_ns: days = mc_cal_extract(&dt, 1000LL * 1000 * 1000 * 60 * 60 * 24); have_days = true; break;
    case MC_DU_ps: days = mc_cal_extract(&dt, 1000LL * 1000 * 1000 * 1000 * 60 * 60 * 24); have_days = true; break;
    default: days = dt < 0 ? -1 : 0; have_days = true; break;  // fs / as: the whole range is within a day of 1970
  }
  if (have_days) mc_cal_ymd_from_days(days, &year, &month, &day);
  int64_t ret;
  if (du == MC_DU_Y) {
    ret = year - 1970;
  } else if (du == MC_DU_M) {
    ret = 12 * (year - 1970) + (month - 1);
  } else {
    const int64_t d = mc_cal_days_from_ymd(year, month, day);
    switch (du) {
      case MC_DU_W: ret = d >= 0 ? d / 7 : (d - 6) / 7; break;
      case MC_DU_D: ret = d; break;
      case MC_DU_h: ret = mc_cal_wrap_mul(d, 24); break;
      case MC_DU_m: ret = mc_cal_wrap_mul(d, 24 * 60); break;
      case MC_DU_s: ret = mc_cal_wrap_mul(d, 24 * 60 * 60); break;
      case MC_DU_ms: ret = mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000); break;
      case MC_DU_us: ret = mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000 * 1000); break;
      case MC_DU_ns: ret = mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000 * 1000 * 1000); break;
      case MC_DU_ps: ret = mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000 * 1000 * 1000 * 1000); break;
      case MC_DU_fs: ret = mc_cal_wrap_mul(mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000 * 1000 * 1000), 1000000); break;
      default: ret = mc_cal_wrap_mul(mc_cal_wrap_mul(d, 24LL * 60 * 60 * 1000 * 1000 * 1000), 1000000000); break;
    }
  }
  if (dn > 1) ret = ret >= 0 ? ret / dn : (ret - dn + 1) / dn;
  return ret;
}
