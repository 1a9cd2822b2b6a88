// Native text front-end: CICIDS2017 featuriser + BERT WordPiece tokenizer.
//
// Replaces two host-side hot spots of the reference:
//  * features_to_text via a row-wise pandas apply (client1.py:68-81, :90);
//  * per-sample, per-epoch pure-Python WordPiece in CICIDS2017Dataset.__getitem__
//    (client1.py:36-50, 2,541 x 16 calls per client), done here once, in a
//    thread-parallel batch, straight into an int32 [N, max_len] id matrix.
//
// Tokenisation follows BERT's BasicTokenizer (lower-case, split on whitespace and
// punctuation) + greedy longest-match-first WordPiece with '##' continuations and
// [UNK] for words longer than 100 chars or with no decomposition.  Input is
// UTF-8; non-ASCII code points are kept as word characters (no accent stripping
// or CJK splitting) -- the featuriser only ever emits ASCII.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "text_core.h"

namespace py = pybind11;
using namespace fdtext;

namespace {

std::vector<const double*> col_ptrs(const std::vector<py::array_t<double, py::array::c_style>>& cols,
                                    size_t& n) {
  if (cols.size() != 10) throw std::runtime_error("render_texts expects 10 columns");
  std::vector<const double*> p;
  n = (size_t)cols[0].size();
  for (auto& c : cols) {
    if ((size_t)c.size() != n) throw std::runtime_error("column length mismatch");
    p.push_back(c.data());
  }
  return p;
}

}  // namespace

PYBIND11_MODULE(_text_native_impl, m) {
  m.doc() = "Native CICIDS2017 featuriser + WordPiece tokenizer";
  m.def("py_repr", [](double v) { std::string s; append_py_repr(s, v); return s; });
  m.def("render_texts",
        [](const std::vector<py::array_t<double, py::array::c_style>>& cols, std::vector<bool> is_int) {
          size_t n;
          auto p = col_ptrs(cols, n);
          std::vector<std::string> out(n);
          {
            py::gil_scoped_release nogil;
            WordPiece::run_parallel(n, 8, [&](size_t lo, size_t hi) {
              for (size_t i = lo; i < hi; ++i) out[i] = render_row(p, is_int, i);
            });
          }
          return out;
        });
  py::class_<WordPiece>(m, "WordPiece")
      .def(py::init<const std::vector<std::string>&, bool, int, int, int, int, int>(),
           py::arg("vocab"), py::arg("lower") = true, py::arg("max_chars") = 100,
           py::arg("unk_id") = 100, py::arg("cls_id") = 101, py::arg("sep_id") = 102,
           py::arg("pad_id") = 0)
      .def("encode", [](const WordPiece& w, const std::string& t, int max_len) {
        return w.encode(t, max_len);
      })
      .def("tokenize", [](const WordPiece& w, const std::string& t) { return w.tokenize_str(t); })
      .def("encode_batch",
           [](const WordPiece& w, const std::vector<std::string>& texts, int max_len, int threads) {
             const size_t n = texts.size();
             py::array_t<int32_t> ids({(py::ssize_t)n, (py::ssize_t)max_len});
             py::array_t<int32_t> lens((py::ssize_t)n);
             int32_t* pid = ids.mutable_data();
             int32_t* plen = lens.mutable_data();
             {
               py::gil_scoped_release nogil;
               w.encode_batch_into(texts, max_len, threads, pid, plen);
             }
             return py::make_tuple(ids, lens);
           },
           py::arg("texts"), py::arg("max_len"), py::arg("threads") = 8)
      .def("featurize_encode",
           [](const WordPiece& w, const std::vector<py::array_t<double, py::array::c_style>>& cols,
              std::vector<bool> is_int, int max_len, int threads) {
             size_t n;
             auto p = col_ptrs(cols, n);
             py::array_t<int32_t> ids({(py::ssize_t)n, (py::ssize_t)max_len});
             py::array_t<int32_t> lens((py::ssize_t)n);
             int32_t* pid = ids.mutable_data();
             int32_t* plen = lens.mutable_data();
             {
               py::gil_scoped_release nogil;
               WordPiece::run_parallel(n, threads, [&](size_t lo, size_t hi) {
                 for (size_t i = lo; i < hi; ++i) {
                   std::vector<int> e = w.encode(render_row(p, is_int, i), max_len);
                   int32_t* row = pid + i * max_len;
                   for (int j = 0; j < max_len; ++j) row[j] = j < (int)e.size() ? e[j] : 0;
                   plen[i] = (int32_t)e.size();
                 }
               });
             }
             return py::make_tuple(ids, lens);
           },
           py::arg("cols"), py::arg("is_int"), py::arg("max_len"), py::arg("threads") = 8);
}
