// Declaration-only subset of Boost.Serialization for the syntax check of
// adapters/orbslam3/ORBmatcher_searches.cc against the reference's headers
// (tests/test_adapter.py): the names their serialize() templates mention
// (never instantiated by the check).  Test infrastructure; it stands in for no
// part of the reference itself.
#pragma once
#include <cstddef>

namespace boost {
namespace serialization {
class access;
template <class Base, class Derived> Base& base_object(Derived& d);
template <class T> class array_wrapper;
template <class T> array_wrapper<T> make_array(T* t, std::size_t s);
template <class T> class nvp;
template <class T> const nvp<T> make_nvp(const char* name, T& t);
template <class Archive, class T> void split_free(Archive& ar, T& t, const unsigned int version);
template <class Archive, class T> void split_member(Archive& ar, T& t, const unsigned int version);
template <class T> struct is_abstract;
}  // namespace serialization
}  // namespace boost

#define BOOST_SERIALIZATION_SPLIT_MEMBER()
#define BOOST_SERIALIZATION_SPLIT_FREE(T)
#define BOOST_SERIALIZATION_ASSUME_ABSTRACT(T)
#define BOOST_CLASS_EXPORT_KEY(T)
#define BOOST_CLASS_EXPORT_IMPLEMENT(T)
#define BOOST_CLASS_EXPORT(T)
#define BOOST_CLASS_EXPORT_GUID(T, K)
#define BOOST_SERIALIZATION_NVP(name) name
