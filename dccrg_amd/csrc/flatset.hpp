// flatset.hpp -- host-side set of cell ids for the AMR bookkeeping (no HIP).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <iterator>
#include <vector>

namespace dccrgx {

// Ascending sort of 64-bit ids: least-significant-digit radix sort over the
// bytes in which the keys differ (ids of a grid span few bytes); std::sort
// for short inputs.
inline void radix_sort_u64(std::vector<uint64_t>& v)
{
    const size_t n = v.size();
    if (n < 4096) {
        std::sort(v.begin(), v.end());
        return;
    }
    uint64_t all_or = 0, all_and = ~0ull;
    for (uint64_t x : v) {
        all_or |= x;
        all_and &= x;
    }
    const uint64_t varying = all_or ^ all_and;
    std::vector<uint64_t> tmp(n);
    uint64_t* a = v.data();
    uint64_t* b = tmp.data();
    for (int sh = 0; sh < 64; sh += 8) {
        if (!((varying >> sh) & 0xff)) continue;
        size_t cnt[257] = {0};
        for (size_t i = 0; i < n; i++) cnt[((a[i] >> sh) & 0xff) + 1]++;
        for (int k = 0; k < 256; k++) cnt[k + 1] += cnt[k];
        for (size_t i = 0; i < n; i++) b[cnt[(a[i] >> sh) & 0xff]++] = a[i];
        std::swap(a, b);
    }
    if (a != v.data()) std::copy(a, a + n, v.data());
}

// A set of nonzero cell ids (0 is error_cell): open addressing, linear
// probing, backward-shift deletion.  The AMR request filters and
// stop_refining do millions of membership tests per adaptive step, which a
// node-based std::set spends in pointer chasing.  Iteration is in table
// order; sorted() gives the ascending ids.
class FlatSet {
  public:
    struct Inserted {
        bool second;
    };
    FlatSet() = default;
    template <class It>
    FlatSet(It b, It e)
    {
        reserve((size_t)std::distance(b, e));
        for (; b != e; ++b) insert(*b);
    }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    void clear()
    {
        std::fill(t_.begin(), t_.end(), 0);
        n_ = 0;
    }
    void reserve(size_t n)
    {
        size_t cap = 16;
        while (cap < 2 * n + 2) cap <<= 1;
        if (cap > t_.size()) rehash(cap);
    }
    size_t count(uint64_t x) const
    {
        if (!n_ || !x) return 0;
        for (size_t i = slot(x);; i = (i + 1) & mask_) {
            if (t_[i] == x) return 1;
            if (!t_[i]) return 0;
        }
    }
    Inserted insert(uint64_t x)
    {
        if (!x) return {false};
        if (2 * (n_ + 1) > t_.size()) rehash(std::max<size_t>(16, 2 * t_.size()));
        for (size_t i = slot(x);; i = (i + 1) & mask_) {
            if (t_[i] == x) return {false};
            if (!t_[i]) {
                t_[i] = x;
                n_++;
                return {true};
            }
        }
    }
    size_t erase(uint64_t x)
    {
        if (!n_ || !x) return 0;
        size_t i = slot(x);
        for (;; i = (i + 1) & mask_) {
            if (!t_[i]) return 0;
            if (t_[i] == x) break;
        }
        // backward shift: move later entries of the probe run into the hole
        size_t j = i;
        for (;;) {
            j = (j + 1) & mask_;
            if (!t_[j]) break;
            const size_t home = slot(t_[j]);
            const bool stays = i <= j ? (i < home && home <= j) : (i < home || home <= j);
            if (stays) continue;
            t_[i] = t_[j];
            i = j;
        }
        t_[i] = 0;
        n_--;
        return 1;
    }
    std::vector<uint64_t> sorted() const
    {
        std::vector<uint64_t> v;
        v.reserve(n_);
        for (uint64_t x : t_)
            if (x) v.push_back(x);
        radix_sort_u64(v);
        return v;
    }
    class const_iterator {
      public:
        const_iterator(const uint64_t* p, const uint64_t* e) : p_(p), e_(e) { skip(); }
        uint64_t operator*() const { return *p_; }
        const_iterator& operator++()
        {
            ++p_;
            skip();
            return *this;
        }
        bool operator!=(const const_iterator& o) const { return p_ != o.p_; }

      private:
        void skip()
        {
            while (p_ != e_ && !*p_) ++p_;
        }
        const uint64_t* p_;
        const uint64_t* e_;
    };
    const_iterator begin() const { return const_iterator(t_.data(), t_.data() + t_.size()); }
    const_iterator end() const { return const_iterator(t_.data() + t_.size(), t_.data() + t_.size()); }

  private:
    size_t slot(uint64_t x) const
    {
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        return (size_t)x & mask_;
    }
    void rehash(size_t cap)
    {
        std::vector<uint64_t> old;
        old.swap(t_);
        t_.assign(cap, 0);
        mask_ = cap - 1;
        n_ = 0;
        for (uint64_t x : old)
            if (x) insert(x);
    }
    std::vector<uint64_t> t_;
    size_t mask_ = 0;
    size_t n_ = 0;
};

// id -> 32-bit value (ghost / retired slots), same table scheme as FlatSet
class FlatMap32 {
  public:
    size_t size() const { return keys_.size() ? n_ : 0; }
    void reserve(size_t n)  // room for n keys without a rehash
    {
        size_t cap = 16;
        while (cap < 2 * n + 2) cap <<= 1;
        if (cap > keys_.size()) rehash(cap);
    }
    size_t count(uint64_t k) const { return find(k) ? 1 : 0; }
    const uint32_t* find(uint64_t k) const
    {
        if (!n_ || !k) return nullptr;
        for (size_t i = slot(k);; i = (i + 1) & mask_) {
            if (keys_[i] == k) return &vals_[i];
            if (!keys_[i]) return nullptr;
        }
    }
    void set(uint64_t k, uint32_t v)  // insert or assign; k != 0
    {
        if (2 * (n_ + 1) > keys_.size()) rehash(std::max<size_t>(16, 2 * keys_.size()));
        for (size_t i = slot(k);; i = (i + 1) & mask_) {
            if (keys_[i] == k) {
                vals_[i] = v;
                return;
            }
            if (!keys_[i]) {
                keys_[i] = k;
                vals_[i] = v;
                n_++;
                return;
            }
        }
    }
    size_t erase(uint64_t k)
    {
        if (!n_ || !k) return 0;
        size_t i = slot(k);
        for (;; i = (i + 1) & mask_) {
            if (!keys_[i]) return 0;
            if (keys_[i] == k) break;
        }
        size_t j = i;
        for (;;) {
            j = (j + 1) & mask_;
            if (!keys_[j]) break;
            const size_t home = slot(keys_[j]);
            const bool stays = i <= j ? (i < home && home <= j) : (i < home || home <= j);
            if (stays) continue;
            keys_[i] = keys_[j];
            vals_[i] = vals_[j];
            i = j;
        }
        keys_[i] = 0;
        n_--;
        return 1;
    }

  private:
    size_t slot(uint64_t x) const
    {
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        return (size_t)x & mask_;
    }
    void rehash(size_t cap)
    {
        std::vector<uint64_t> ok;
        std::vector<uint32_t> ov;
        ok.swap(keys_);
        ov.swap(vals_);
        keys_.assign(cap, 0);
        vals_.assign(cap, 0);
        mask_ = cap - 1;
        n_ = 0;
        for (size_t i = 0; i < ok.size(); i++)
            if (ok[i]) set(ok[i], ov[i]);
    }
    std::vector<uint64_t> keys_;
    std::vector<uint32_t> vals_;
    size_t mask_ = 0;
    size_t n_ = 0;
};

}  // namespace dccrgx
