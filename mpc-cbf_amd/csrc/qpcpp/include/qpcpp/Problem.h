// qpcpp/Problem.h — header-only host mirror of the reference's qpcpp problem container
// (interface: workspace/lib/qpcpp/include/qpcpp/Problem.h; behaviour: src/Problem.cpp), written
// for this repository so the HIPSolver adapter and its tests build without the reference tree.
// Same public names, argument meaning, iteration order and error behaviour:
//   - variables / constraints live in forward_lists filled with push_front, so iteration visits
//     them newest first (Problem.cpp:208,228) and pointers stay valid;
//   - addVariable / addLinearConstraint default to [lowest(), max()] (= unbounded);
//   - quadratic coefficients are stored once per unordered pair and accumulate (Problem.cpp:101-116):
//     the objective is sum_{i<=j} q_ij x_i x_j + sum c_i x_i + constant, no 1/2 factor;
//   - touching a variable of another problem throws std::runtime_error.
#pragma once

#include <cstddef>
#include <forward_list>
#include <functional>
#include <limits>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>

namespace qpcpp {

template <typename T>
class Problem;

namespace detail {
template <typename T>
struct Key {  // only Problem<T> can construct variables and constraints
  private:
    Key() = default;
    friend class Problem<T>;
};
[[noreturn]] inline void unknown_variable(const char* where) {
    throw std::runtime_error(std::string(where) + ": variable does not exist in the problem");
}
}  // namespace detail

template <typename T>
class Variable {
  public:
    Variable(detail::Key<T>, const Problem<T>& owner, T lo, T hi) : owner_(&owner), lo_(lo), hi_(hi) {}
    const Problem<T>& context_problem() const { return *owner_; }
    T min() const { return lo_; }
    T max() const { return hi_; }
    void set_min(T v) { lo_ = v; }
    void set_max(T v) { hi_ = v; }
    T solution_value() const { return value_; }
    void set_solution_value(T v) { value_ = v; }

  private:
    const Problem<T>* owner_;
    T lo_, hi_;
    T value_ = T(0);
};

template <typename T>
class LinearConstraint {
  public:
    LinearConstraint(detail::Key<T>, const Problem<T>& owner, T lo, T hi) : owner_(&owner), lo_(lo), hi_(hi) {}
    void setCoefficient(const Variable<T>* v, T coefficient);
    T getCoefficient(const Variable<T>* v) const;
    T min() const { return lo_; }
    T max() const { return hi_; }

  private:
    const Problem<T>* owner_;
    T lo_, hi_;
    std::unordered_map<const Variable<T>*, T> coef_;
};

template <typename T>
class CostFunction {
  public:
    explicit CostFunction(const Problem<T>& owner) : owner_(&owner) {}
    void addQuadraticTerm(const Variable<T>* a, const Variable<T>* b, T coefficient);
    T getQuadraticCoefficient(const Variable<T>* a, const Variable<T>* b) const;
    void addLinearTerm(const Variable<T>* v, T coefficient);
    T getLinearCoefficient(const Variable<T>* v) const;
    void add_constant(T v) { constant_ += v; }
    T constant() const { return constant_; }
    void setZero() {
        quad_.clear();
        lin_.clear();
        constant_ = T(0);
    }

  private:
    using Pair = std::pair<const Variable<T>*, const Variable<T>*>;
    struct PairHash {
        std::size_t operator()(const Pair& p) const {
            const std::size_t h = std::hash<const void*>()(p.first);
            return h ^ (std::hash<const void*>()(p.second) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2));
        }
    };
    static Pair ordered(const Variable<T>* a, const Variable<T>* b) {
        return std::less<const Variable<T>*>()(b, a) ? Pair(b, a) : Pair(a, b);
    }
    const Problem<T>* owner_;
    std::unordered_map<Pair, T, PairHash> quad_;
    std::unordered_map<const Variable<T>*, T> lin_;
    T constant_ = T(0);
};

template <typename T>
class Problem {
  public:
    using Variable = qpcpp::Variable<T>;
    using LinearConstraint = qpcpp::LinearConstraint<T>;
    using CostFunction = qpcpp::CostFunction<T>;

    Problem() : cost_(*this) {}
    Problem(const Problem&) = delete;
    Problem& operator=(const Problem&) = delete;

    std::size_t numVariables() const { return n_vars_; }
    Variable* addVariable(T min = std::numeric_limits<T>::lowest(), T max = std::numeric_limits<T>::max()) {
        vars_.emplace_front(detail::Key<T>(), *this, min, max);
        Variable* v = &vars_.front();
        known_.insert(v);
        ++n_vars_;
        return v;
    }
    bool hasVariable(const Variable* v) const { return known_.count(v) != 0; }
    std::size_t numLinearConstraints() const { return n_rows_; }
    LinearConstraint* addLinearConstraint(T min = std::numeric_limits<T>::lowest(),
                                          T max = std::numeric_limits<T>::max()) {
        rows_.emplace_front(detail::Key<T>(), *this, min, max);
        ++n_rows_;
        return &rows_.front();
    }
    const std::forward_list<Variable>& variables() const { return vars_; }
    const std::forward_list<LinearConstraint>& linear_constraints() const { return rows_; }
    CostFunction* cost_function() { return &cost_; }
    void clearLinearConstraints() {
        rows_.clear();
        n_rows_ = 0;
    }
    void setCostFunctionToZero() { cost_.setZero(); }
    // clears cost and rows; variables (and their bounds) persist (Problem.cpp:256-270)
    void resetProblem() {
        setCostFunctionToZero();
        clearLinearConstraints();
    }

  private:
    std::forward_list<Variable> vars_;
    std::unordered_set<const Variable*> known_;
    std::size_t n_vars_ = 0;
    std::forward_list<LinearConstraint> rows_;
    std::size_t n_rows_ = 0;
    CostFunction cost_;
};

template <typename T>
void LinearConstraint<T>::setCoefficient(const Variable<T>* v, T coefficient) {
    if (!owner_->hasVariable(v)) detail::unknown_variable("LinearConstraint::setCoefficient");
    coef_[v] = coefficient;  // overwrite, not accumulate
}

template <typename T>
T LinearConstraint<T>::getCoefficient(const Variable<T>* v) const {
    if (!owner_->hasVariable(v)) detail::unknown_variable("LinearConstraint::getCoefficient");
    const auto it = coef_.find(v);
    return it == coef_.end() ? T(0) : it->second;
}

template <typename T>
void CostFunction<T>::addQuadraticTerm(const Variable<T>* a, const Variable<T>* b, T coefficient) {
    if (!owner_->hasVariable(a) || !owner_->hasVariable(b)) detail::unknown_variable("CostFunction::addQuadraticTerm");
    quad_[ordered(a, b)] += coefficient;
}

template <typename T>
T CostFunction<T>::getQuadraticCoefficient(const Variable<T>* a, const Variable<T>* b) const {
    if (!owner_->hasVariable(a) || !owner_->hasVariable(b))
        detail::unknown_variable("CostFunction::getQuadraticCoefficient");
    const auto it = quad_.find(ordered(a, b));
    return it == quad_.end() ? T(0) : it->second;
}

template <typename T>
void CostFunction<T>::addLinearTerm(const Variable<T>* v, T coefficient) {
    if (!owner_->hasVariable(v)) detail::unknown_variable("CostFunction::addLinearTerm");
    lin_[v] += coefficient;
}

template <typename T>
T CostFunction<T>::getLinearCoefficient(const Variable<T>* v) const {
    if (!owner_->hasVariable(v)) detail::unknown_variable("CostFunction::getLinearCoefficient");
    const auto it = lin_.find(v);
    return it == lin_.end() ? T(0) : it->second;
}

}  // namespace qpcpp
