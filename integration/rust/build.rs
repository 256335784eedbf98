// build.rs for the reference crate (next to Cargo.toml): link the lib crate against librtw.so.
// RTW_LIB_DIR names the directory holding librtw.so (this repository builds it in
// raytracinginaweekend_amd/); at run time the loader finds it through LD_LIBRARY_PATH or an rpath.
fn main() {
    let dir = std::env::var("RTW_LIB_DIR").unwrap_or_else(|_| "../raytracinginaweekend_amd".to_string());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=rtw");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=RTW_LIB_DIR");
}
