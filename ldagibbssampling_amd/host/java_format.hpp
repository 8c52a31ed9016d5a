// java_format.hpp — the two number renderings Mallet's text outputs use.
//
//  java_double(x)      Double.toString(x): shortest round-trip digits (the
//                      JDK >= 19 algorithm; older JDKs occasionally print one
//                      more digit), plain notation for 1e-3 <= |x| < 1e7, else
//                      "d.dddE<exp>"; always at least one fraction digit.
//                      Used by printDocumentTopics' weights (string
//                      concatenation of a double).
//  java_number5(x)     NumberFormat.getInstance() (US locale) with
//                      setMaximumFractionDigits(5): HALF_EVEN on the exact
//                      binary value, trailing zeros dropped, "," grouping.
//                      Mallet's ParallelTopicModel.formatter (alpha in
//                      printTopWords, LL/token in the estimate() log).
#pragma once
#include <string>

namespace lda_host {

std::string java_double(double x);
std::string java_number5(double x);

}  // namespace lda_host
