// A vector of trivially copyable elements that keeps up to N of them inside the object and
// moves to the heap only beyond that (the role of reference src/prevector.h, the storage of
// CScript). Almost every script on the chain is a P2PKH / P2SH / P2PK output script of 23-35
// bytes; inline storage makes a Coin or a CTxOut one allocation-free object, which is what the
// parallel UTXO pass copies, moves and frees ~100k times per 8 MB block.
//
// Layout (packed, 4 + max(N, 12) bytes): a 32-bit word holding the size with the top bit set
// while the elements live on the heap, then either the N inline elements or the heap pointer and
// capacity. Iterators are plain pointers; any growth may move the elements (like std::vector).
#pragma once
#include <algorithm>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <iterator>
#include <new>
#include <type_traits>

namespace bcp {

template <unsigned N, typename T> class prevector {
    static_assert(std::is_trivially_copyable<T>::value, "prevector holds trivially copyable elements");
    static constexpr uint32_t HEAP = 0x80000000u;

public:
    typedef T value_type;
    typedef uint32_t size_type;
    typedef std::ptrdiff_t difference_type;
    typedef T& reference;
    typedef const T& const_reference;
    typedef T* pointer;
    typedef const T* const_pointer;
    typedef T* iterator;
    typedef const T* const_iterator;
    typedef std::reverse_iterator<iterator> reverse_iterator;
    typedef std::reverse_iterator<const_iterator> const_reverse_iterator;

    prevector() : meta(0) {}
    explicit prevector(size_type n) : meta(0) { resize(n); }
    prevector(size_type n, const T& v) : meta(0) { assign(n, v); }
    template <typename It, typename = typename std::iterator_traits<It>::iterator_category>
    prevector(It first, It last) : meta(0) {
        assign(first, last);
    }
    prevector(std::initializer_list<T> il) : meta(0) { assign(il.begin(), il.end()); }
    prevector(const prevector& o) : meta(0) { assign(o.begin(), o.end()); }
    prevector(prevector&& o) noexcept : meta(o.meta) {
        std::memcpy(&u, &o.u, sizeof(u));
        o.meta = 0;
    }
    ~prevector() {
        if (is_heap()) std::free(u.h.p);
    }
    prevector& operator=(const prevector& o) {
        if (this != &o) assign(o.begin(), o.end());
        return *this;
    }
    prevector& operator=(prevector&& o) noexcept {
        if (this != &o) {
            if (is_heap()) std::free(u.h.p);
            meta = o.meta;
            std::memcpy(&u, &o.u, sizeof(u));
            o.meta = 0;
        }
        return *this;
    }

    size_type size() const { return meta & ~HEAP; }
    bool empty() const { return size() == 0; }
    size_type capacity() const { return is_heap() ? u.h.cap : N; }
    static constexpr size_type max_size() { return HEAP - 1; }

    T* data() { return is_heap() ? u.h.p : u.d; }
    const T* data() const { return is_heap() ? u.h.p : u.d; }
    iterator begin() { return data(); }
    const_iterator begin() const { return data(); }
    const_iterator cbegin() const { return data(); }
    iterator end() { return data() + size(); }
    const_iterator end() const { return data() + size(); }
    const_iterator cend() const { return data() + size(); }
    reverse_iterator rbegin() { return reverse_iterator(end()); }
    const_reverse_iterator rbegin() const { return const_reverse_iterator(end()); }
    reverse_iterator rend() { return reverse_iterator(begin()); }
    const_reverse_iterator rend() const { return const_reverse_iterator(begin()); }
    T& operator[](size_type i) { return data()[i]; }
    const T& operator[](size_type i) const { return data()[i]; }
    T& front() { return data()[0]; }
    const T& front() const { return data()[0]; }
    T& back() { return data()[size() - 1]; }
    const T& back() const { return data()[size() - 1]; }

    void reserve(size_type n) {
        if (n > capacity()) grow_to(n);
    }
    void shrink_to_fit() {
        const size_type n = size();
        if (!is_heap() || n == u.h.cap) return;
        if (n <= N) {
            T* p = u.h.p;
            std::memcpy(u.d, p, n * sizeof(T));
            std::free(p);
            meta = n;
        } else {
            grow_exact(n);
        }
    }
    void clear() { set_size(0); }
    void resize(size_type n) {
        const size_type s = size();
        if (n > s) {
            reserve(n);
            std::memset(data() + s, 0, (n - s) * sizeof(T));
        }
        set_size(n);
    }
    void resize(size_type n, const T& v) {
        const size_type s = size();
        if (n > s) {
            reserve(n);
            std::fill(data() + s, data() + n, v);
        }
        set_size(n);
    }
    void assign(size_type n, const T& v) {
        clear();
        resize(n, v);
    }
    template <typename It> void assign(It first, It last) {
        const size_type n = (size_type)std::distance(first, last);
        clear();
        reserve(n);
        std::copy(first, last, data());
        set_size(n);
    }
    void push_back(const T& v) {
        const size_type s = size();
        if (s == capacity()) {
            const T copy = v; // v may live in this vector
            grow_to(s + 1);
            data()[s] = copy;
        } else {
            data()[s] = v;
        }
        set_size(s + 1);
    }
    void emplace_back(const T& v) { push_back(v); }
    void pop_back() { set_size(size() - 1); }

    iterator insert(const_iterator pos, const T& v) {
        const T copy = v;
        const size_type at = (size_type)(pos - begin());
        open_gap(at, 1);
        data()[at] = copy;
        return begin() + at;
    }
    iterator insert(const_iterator pos, size_type n, const T& v) {
        const T copy = v;
        const size_type at = (size_type)(pos - begin());
        open_gap(at, n);
        std::fill(data() + at, data() + at + n, copy);
        return begin() + at;
    }
    template <typename It, typename = typename std::iterator_traits<It>::iterator_category>
    iterator insert(const_iterator pos, It first, It last) {
        const size_type at = (size_type)(pos - begin());
        const size_type n = (size_type)std::distance(first, last);
        if (n == 0) return begin() + at;
        // the source may alias this vector: copy it out before the gap moves it
        if (aliases(first, last)) {
            prevector tmp(first, last);
            return insert(pos, tmp.begin(), tmp.end());
        }
        open_gap(at, n);
        std::copy(first, last, data() + at);
        return begin() + at;
    }
    iterator erase(const_iterator pos) { return erase(pos, pos + 1); }
    iterator erase(const_iterator first, const_iterator last) {
        const size_type a = (size_type)(first - begin()), b = (size_type)(last - begin()), s = size();
        std::memmove(data() + a, data() + b, (s - b) * sizeof(T));
        set_size(s - (b - a));
        return begin() + a;
    }
    void swap(prevector& o) noexcept {
        prevector t(std::move(o));
        o = std::move(*this);
        *this = std::move(t);
    }

    // heap bytes held (memory accounting)
    size_t allocated_memory() const { return is_heap() ? (size_t)u.h.cap * sizeof(T) : 0; }

    friend bool operator==(const prevector& a, const prevector& b) {
        return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0;
    }
    friend bool operator!=(const prevector& a, const prevector& b) { return !(a == b); }
    friend bool operator<(const prevector& a, const prevector& b) {
        return std::lexicographical_compare(a.begin(), a.end(), b.begin(), b.end());
    }

private:
    bool is_heap() const { return (meta & HEAP) != 0; }
    void set_size(size_type n) { meta = (meta & HEAP) | n; }
    template <typename It> bool aliases(It first, It last) const {
        if constexpr (std::is_pointer<It>::value) {
            const T* f = &*first;
            return f >= data() && f < data() + capacity() && first != last;
        } else {
            return false;
        }
    }
    // capacity for at least n, growing by half again (like the common vector policies)
    void grow_to(size_type n) {
        size_type c = capacity();
        c = c + c / 2;
        grow_exact(std::max(n, c));
    }
    void grow_exact(size_type cap) {
        const size_type s = size();
        T* p = static_cast<T*>(std::malloc((size_t)cap * sizeof(T)));
        if (!p) throw std::bad_alloc();
        std::memcpy(p, data(), s * sizeof(T));
        if (is_heap()) std::free(u.h.p);
        u.h.p = p;
        u.h.cap = cap;
        meta = HEAP | s;
    }
    void open_gap(size_type at, size_type n) {
        const size_type s = size();
        reserve(s + n);
        std::memmove(data() + at + n, data() + at, (s - at) * sizeof(T));
        set_size(s + n);
    }

    uint32_t meta;
    union Storage {
        T d[N];
        struct __attribute__((packed)) {
            T* p;
            uint32_t cap;
        } h;
    } __attribute__((packed)) u;
} __attribute__((packed));

} // namespace bcp
