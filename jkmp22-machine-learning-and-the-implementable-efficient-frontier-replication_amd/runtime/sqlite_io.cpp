// Columnar SQLite reader / writer for the panel stages (SURVEY §2.2 "SQLite I/O").
//
// The reference moves its panels through SQLite with pandas (read_sql_query / to_sql:
// Prepare_Data.py:105-110, 487-489; PFML_Input_Data.py:53-79).  pandas materialises every
// value as a Python object and back (at the production shape - 430k rows x 130 columns of
// Factors / Factors_processed - 23 s to read and 18 s to write one table, three quarters of
// the S2 stage).  Here a query is stepped once in C++ and each result column lands in a
// typed buffer (int64, float64 with NaN for NULL, or text bytes + offsets); the writer binds
// typed column buffers into one prepared INSERT inside one transaction.  Same SQL, same
// schema (pandas' SQLite type names), same values; Python builds the DataFrame from the
// column buffers (data/io.py).
//
// libsqlite3 ships without its header in this image, so the few C-API entry points used are
// declared here (stable SQLite 3 ABI) and the library is linked as libsqlite3.so.0.
#include <omp.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
struct sqlite3;
struct sqlite3_stmt;
int sqlite3_open_v2(const char*, sqlite3**, int, const char*);
int sqlite3_close(sqlite3*);
int sqlite3_prepare_v2(sqlite3*, const char*, int, sqlite3_stmt**, const char**);
int sqlite3_step(sqlite3_stmt*);
int sqlite3_reset(sqlite3_stmt*);
int sqlite3_finalize(sqlite3_stmt*);
int sqlite3_column_count(sqlite3_stmt*);
const char* sqlite3_column_name(sqlite3_stmt*, int);
int sqlite3_column_type(sqlite3_stmt*, int);
long long sqlite3_column_int64(sqlite3_stmt*, int);
double sqlite3_column_double(sqlite3_stmt*, int);
const unsigned char* sqlite3_column_text(sqlite3_stmt*, int);
int sqlite3_column_bytes(sqlite3_stmt*, int);
int sqlite3_bind_int64(sqlite3_stmt*, int, long long);
int sqlite3_bind_double(sqlite3_stmt*, int, double);
int sqlite3_bind_text(sqlite3_stmt*, int, const char*, int, void (*)(void*));
int sqlite3_bind_null(sqlite3_stmt*, int);
int sqlite3_exec(sqlite3*, const char*, int (*)(void*, int, char**, char**), void*, char**);
const char* sqlite3_errmsg(sqlite3*);
}

namespace {

constexpr int SQ_OK = 0, SQ_ROW = 100, SQ_DONE = 101;
constexpr int SQ_INTEGER = 1, SQ_FLOAT = 2, SQ_TEXT = 3, SQ_NULL = 5;
constexpr int OPEN_READONLY = 0x1, OPEN_READWRITE = 0x2, OPEN_CREATE = 0x4;
void (*const SQ_TRANSIENT)(void*) = reinterpret_cast<void (*)(void*)>(-1);

// Result column kinds handed to Python (pandas' inference over the returned Python values):
//   1 int64 (only integers, no NULL), 2 float64 (numbers, NULL -> NaN), 3 text (NULL kept),
//   0 all NULL, -1 mixed text / numbers (the caller falls back to pandas)
struct Col {
  bool has_int = false, has_real = false, has_text = false, has_null = false;
  std::vector<double> d;
  std::vector<long long> i;
  std::vector<unsigned char> isnull;
  std::string text;
  std::vector<long long> off{0};
  int kind() const {
    if (has_text && (has_int || has_real)) return -1;
    if (has_text) return 3;
    if (has_real || (has_int && has_null)) return 2;
    if (has_int) return 1;
    return 0;
  }
};

struct Result {
  std::vector<std::string> names;
  std::vector<Col> cols;
  long long nrow = 0;
  std::string err;
};

void set_err(char* err, int errlen, const std::string& msg) {
  if (err && errlen > 0) {
    std::strncpy(err, msg.c_str(), errlen - 1);
    err[errlen - 1] = 0;
  }
}


// step `sql` on `con` into R (columns appended); false on a SQLite error (message in R->err)
bool run_query(sqlite3* con, const std::string& sql, Result* R) {
  sqlite3_stmt* st = nullptr;
  if (sqlite3_prepare_v2(con, sql.c_str(), -1, &st, nullptr) != SQ_OK) {
    R->err = sqlite3_errmsg(con);
    return false;
  }
  const int nc = sqlite3_column_count(st);
  R->cols.resize(nc);
  R->names.clear();
  for (int c = 0; c < nc; ++c) R->names.emplace_back(sqlite3_column_name(st, c));
  int rc;
  while ((rc = sqlite3_step(st)) == SQ_ROW) {
    for (int c = 0; c < nc; ++c) {
      Col& col = R->cols[c];
      const int t = sqlite3_column_type(st, c);
      double dv = NAN;
      long long iv = 0;
      unsigned char nul = 0;
      if (t == SQ_INTEGER) {
        iv = sqlite3_column_int64(st, c);
        dv = (double)iv;
        col.has_int = true;
      } else if (t == SQ_FLOAT) {
        dv = sqlite3_column_double(st, c);
        iv = (long long)dv;
        col.has_real = true;
      } else if (t == SQ_TEXT) {
        const unsigned char* s = sqlite3_column_text(st, c);
        const int nb = sqlite3_column_bytes(st, c);
        col.text.append(reinterpret_cast<const char*>(s), nb);
        col.has_text = true;
      } else {
        nul = 1;
        col.has_null = true;
      }
      col.d.push_back(dv);
      col.i.push_back(iv);
      col.isnull.push_back(nul);
      col.off.push_back((long long)col.text.size());
    }
    ++R->nrow;
  }
  const bool ok = rc == SQ_DONE;
  if (!ok) R->err = sqlite3_errmsg(con);
  sqlite3_finalize(st);
  return ok;
}

// "SELECT <columns> FROM <table>" with nothing after the table name -> the table name (the
// query is then read in rowid ranges by several connections at once), else ""
std::string plain_scan_table(const std::string& sql) {
  std::string u(sql);
  for (auto& ch : u) ch = (char)std::toupper((unsigned char)ch);
  if (u.compare(0, 7, "SELECT ") != 0) return "";
  const size_t f = u.rfind(" FROM ");
  if (f == std::string::npos) return "";
  size_t a = f + 6;
  while (a < sql.size() && sql[a] == ' ') ++a;
  size_t b = sql.size();
  while (b > a && (sql[b - 1] == ' ' || sql[b - 1] == ';')) --b;
  const std::string t = sql.substr(a, b - a);
  if (t.empty()) return "";
  for (char ch : t)
    if (!(std::isalnum((unsigned char)ch) || ch == '_')) return "";
  for (const char* kw : {" WHERE ", " JOIN ", " GROUP ", " ORDER ", " LIMIT ", " UNION "})
    if (u.find(kw) != std::string::npos) return "";
  // the select list must be `*` or plain column names (optionally "quoted"): DISTINCT,
  // aggregates and expressions (count(*), max(eom), a + b) give per-part rows that do not
  // concatenate to the query's result, so they run on one connection
  const std::string list = sql.substr(7, f - 7);
  size_t s0 = list.find_first_not_of(' ');
  if (s0 == std::string::npos) return "";
  const std::string lt = list.substr(s0, list.find_last_not_of(' ') - s0 + 1);
  if (lt == "*") return t;
  std::string ul(lt);
  for (auto& ch : ul) ch = (char)std::toupper((unsigned char)ch);
  if (ul.compare(0, 9, "DISTINCT ") == 0 || ul.compare(0, 4, "ALL ") == 0) return "";
  size_t p = 0;
  while (p <= lt.size()) {
    size_t q = lt.find(',', p);
    if (q == std::string::npos) q = lt.size();
    std::string tok = lt.substr(p, q - p);
    const size_t a0 = tok.find_first_not_of(' '), a1 = tok.find_last_not_of(' ');
    if (a0 == std::string::npos) return "";
    tok = tok.substr(a0, a1 - a0 + 1);
    if (tok.size() >= 2 && tok.front() == '"' && tok.back() == '"') {
      for (size_t k = 1; k + 1 < tok.size(); ++k)
        if (tok[k] == '"') return "";
    } else {
      for (char ch : tok)
        if (!(std::isalnum((unsigned char)ch) || ch == '_')) return "";
    }
    p = q + 1;
  }
  return t;
}

}  // namespace

// Run a query; plain full-table scans are split into rowid ranges read by up to
// omp_get_max_threads() connections in parallel and concatenated in rowid order (the order
// of the plain scan).  Anything else, or a table without rowid, runs on one connection.
extern "C" void* pfml_sql_query(const char* db, const char* sql, long long* nrow, int* ncol,
                                char* err, int errlen) {
  sqlite3* con = nullptr;
  if (sqlite3_open_v2(db, &con, OPEN_READONLY, nullptr) != SQ_OK) {
    set_err(err, errlen, con ? sqlite3_errmsg(con) : "open failed");
    if (con) sqlite3_close(con);
    return nullptr;
  }
  auto* R = new Result;
  const std::string table = plain_scan_table(sql);
  long long lo = 0, hi = -1;
  int parts = 1;
  if (!table.empty()) {
    Result mm;
    if (run_query(con, "SELECT min(rowid), max(rowid), count(*) FROM \"" + table + "\"", &mm) &&
        mm.nrow == 1 && mm.cols.size() == 3 && mm.cols[0].has_int && mm.cols[2].i[0] > 65536) {
      lo = mm.cols[0].i[0];
      hi = mm.cols[1].i[0];
      parts = std::max(1, std::min(omp_get_max_threads(), 16));
    }
  }
  bool ok;
  if (parts == 1) {
    ok = run_query(con, sql, R);
    if (!ok) set_err(err, errlen, R->err);
  } else {
    std::vector<Result> P(parts);
    std::vector<int> good(parts, 0);
    const long long span = hi - lo + 1;
#pragma omp parallel for num_threads(parts) schedule(static, 1)
    for (int k = 0; k < parts; ++k) {
      const long long a = lo + span * k / parts, b = lo + span * (k + 1) / parts - 1;
      sqlite3* ck = nullptr;
      if (sqlite3_open_v2(db, &ck, OPEN_READONLY, nullptr) == SQ_OK) {
        good[k] = run_query(ck, std::string(sql) + " WHERE rowid BETWEEN " + std::to_string(a) +
                                    " AND " + std::to_string(b) + " ORDER BY rowid",
                            &P[k]);
      } else {
        P[k].err = "open failed";
      }
      if (ck) sqlite3_close(ck);
    }
    ok = true;
    for (int k = 0; k < parts; ++k)
      if (!good[k]) {
        ok = false;
        set_err(err, errlen, P[k].err);
      }
    if (ok) {
      R->names = P[0].names;
      R->cols.resize(P[0].cols.size());
      for (size_t c = 0; c < R->cols.size(); ++c) {
        Col& o = R->cols[c];
        size_t n = 0, nb = 0;
        for (int k = 0; k < parts; ++k) {
          n += P[k].cols.size() > c ? P[k].cols[c].d.size() : 0;
          nb += P[k].cols.size() > c ? P[k].cols[c].text.size() : 0;
        }
        o.d.reserve(n);
        o.i.reserve(n);
        o.isnull.reserve(n);
        o.off.reserve(n + 1);
        o.text.reserve(nb);
        for (int k = 0; k < parts; ++k) {
          if (P[k].cols.size() <= c) continue;       // (an empty part still has its columns)
          const Col& s = P[k].cols[c];
          o.has_int |= s.has_int;
          o.has_real |= s.has_real;
          o.has_text |= s.has_text;
          o.has_null |= s.has_null;
          o.d.insert(o.d.end(), s.d.begin(), s.d.end());
          o.i.insert(o.i.end(), s.i.begin(), s.i.end());
          o.isnull.insert(o.isnull.end(), s.isnull.begin(), s.isnull.end());
          const long long base = (long long)o.text.size();
          for (size_t r = 1; r < s.off.size(); ++r) o.off.push_back(base + s.off[r]);
          o.text += s.text;
        }
      }
      for (int k = 0; k < parts; ++k) R->nrow += P[k].nrow;
    }
  }
  sqlite3_close(con);
  if (!ok) {
    delete R;
    return nullptr;
  }
  *nrow = R->nrow;
  *ncol = (int)R->names.size();
  return R;
}

extern "C" const char* pfml_sql_col_name(void* h, int c) {
  return static_cast<Result*>(h)->names[c].c_str();
}
extern "C" int pfml_sql_col_kind(void* h, int c) { return static_cast<Result*>(h)->cols[c].kind(); }
extern "C" void pfml_sql_col_f64(void* h, int c, double* out) {
  const Col& col = static_cast<Result*>(h)->cols[c];
  std::memcpy(out, col.d.data(), col.d.size() * sizeof(double));
}
extern "C" void pfml_sql_col_i64(void* h, int c, long long* out) {
  const Col& col = static_cast<Result*>(h)->cols[c];
  std::memcpy(out, col.i.data(), col.i.size() * sizeof(long long));
}
extern "C" long long pfml_sql_col_text_bytes(void* h, int c) {
  return (long long)static_cast<Result*>(h)->cols[c].text.size();
}
// text bytes, nrow + 1 offsets, and the NULL mask
extern "C" void pfml_sql_col_text(void* h, int c, char* buf, long long* off, unsigned char* isnull) {
  const Col& col = static_cast<Result*>(h)->cols[c];
  std::memcpy(buf, col.text.data(), col.text.size());
  std::memcpy(off, col.off.data(), col.off.size() * sizeof(long long));
  std::memcpy(isnull, col.isnull.data(), col.isnull.size());
}
extern "C" void pfml_sql_free(void* h) { delete static_cast<Result*>(h); }

// Write a table from column buffers (pandas DataFrame.to_sql(index=False) semantics):
//   kinds[c]: 1 int64, 2 float64 (NaN -> NULL), 3 text (offsets[c]: nrow + 1 byte offsets,
//   nulls[c]: per-row NULL flags or null), 4 bool (stored 0 / 1)
//   decl[c]:  the SQL column type (pandas' names: INTEGER, REAL, TEXT, TIMESTAMP)
//   replace:  1 = DROP + CREATE (if_exists="replace"), 0 = CREATE IF NOT EXISTS + append
extern "C" int pfml_sql_write(const char* db, const char* table, int replace, int ncol,
                              const char** names, const char** decl, const int* kinds,
                              const void** data, const long long** offsets,
                              const unsigned char** nulls, long long nrow, char* err,
                              int errlen) {
  sqlite3* con = nullptr;
  if (sqlite3_open_v2(db, &con, OPEN_READWRITE | OPEN_CREATE, nullptr) != SQ_OK) {
    set_err(err, errlen, con ? sqlite3_errmsg(con) : "open failed");
    if (con) sqlite3_close(con);
    return 1;
  }
  auto q = [](const std::string& s) {       // SQL identifier quoting, as pandas does
    std::string o = "\"";
    for (char ch : s) {
      if (ch == '"') o += '"';
      o += ch;
    }
    return o + "\"";
  };
  std::string sql;
  auto exec = [&](const std::string& s) {
    char* msg = nullptr;
    if (sqlite3_exec(con, s.c_str(), nullptr, nullptr, &msg) != SQ_OK) {
      set_err(err, errlen, sqlite3_errmsg(con));
      return false;
    }
    return true;
  };
  bool ok = exec("PRAGMA synchronous=OFF") && exec("BEGIN");
  if (ok && replace) ok = exec("DROP TABLE IF EXISTS " + q(table));
  if (ok) {
    sql = "CREATE TABLE IF NOT EXISTS " + q(table) + " (";
    for (int c = 0; c < ncol; ++c) sql += (c ? ", " : "") + q(names[c]) + " " + decl[c];
    sql += ")";
    ok = exec(sql);
  }
  sqlite3_stmt* st = nullptr;
  if (ok) {
    sql = "INSERT INTO " + q(table) + " VALUES (";
    for (int c = 0; c < ncol; ++c) sql += c ? ", ?" : "?";
    sql += ")";
    if (sqlite3_prepare_v2(con, sql.c_str(), -1, &st, nullptr) != SQ_OK) {
      set_err(err, errlen, sqlite3_errmsg(con));
      ok = false;
    }
  }
  for (long long r = 0; ok && r < nrow; ++r) {
    for (int c = 0; c < ncol; ++c) {
      const int k = kinds[c];
      if (k == 1 || k == 4) {
        sqlite3_bind_int64(st, c + 1, static_cast<const long long*>(data[c])[r]);
      } else if (k == 2) {
        const double v = static_cast<const double*>(data[c])[r];
        if (std::isnan(v)) sqlite3_bind_null(st, c + 1);
        else sqlite3_bind_double(st, c + 1, v);
      } else {
        if (nulls[c] && nulls[c][r]) {
          sqlite3_bind_null(st, c + 1);
        } else {
          const long long a = offsets[c][r], b = offsets[c][r + 1];
          sqlite3_bind_text(st, c + 1, static_cast<const char*>(data[c]) + a, (int)(b - a),
                            SQ_TRANSIENT);
        }
      }
    }
    if (sqlite3_step(st) != SQ_DONE) {
      set_err(err, errlen, sqlite3_errmsg(con));
      ok = false;
    }
    sqlite3_reset(st);
  }
  if (st) sqlite3_finalize(st);
  ok = ok && exec("COMMIT");
  if (!ok) exec("ROLLBACK");
  sqlite3_close(con);
  return ok ? 0 : 1;
}
