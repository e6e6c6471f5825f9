//! The vote-batching ingress at `Consensus::proc_network_msg` (reference consensus.rs:210-262;
//! SURVEY.md 8(f) row 1): the Rust form of `consensus_overlord_amd/ingress.py` (`VoteIngress`),
//! the same state machine.
//!
//! The reference decodes each network message and hands it to overlord at once; overlord then
//! calls `Crypto::verify_signature` once per `SignedVote` / `SignedChoke`, serially. This shim
//! holds the decoded votes and chokes of a (height, round, kind) group, verifies everything held
//! as ONE device batch (`HipCrypto::prefetch` -> `ovh_prefetch`: RLC batch check + exact per-vote
//! codes into the library's verdict cache) and only then forwards the messages to overlord, in
//! arrival order. overlord's serial `verify_signature` calls on them are verdict-cache hits.
//!
//! Flush policy: a group that reaches `batch_size` flushes everything held; the default is what
//! one round brings over the network -- the validator count minus one when this node is a
//! validator (its own vote never crosses the network, consensus.rs:721-771), else the validator
//! count. A deadline flushes the rest: every arrival checks it, and `poll` (driven by the node's
//! tokio interval) flushes a group that stopped growing once its oldest message has waited
//! `max_delay`. `AggregatedVote` and `SignedProposal` are not batched; they first flush what is
//! held. A message that does not decode is dropped with a warning, as the reference does.
//!
//! The signed bytes: hash(rlp(Vote)) for a vote (on the device: `ovh_vote_digests`, rlp + SM3),
//! hash(rlp([height, round])) for a choke (overlord `HashChoke`).
use crate::{ffi, HipCrypto};
use bytes::Bytes;
use overlord::types::{AggregatedVote, OverlordMsg, SignedChoke, SignedProposal, SignedVote};
use overlord::Codec;
use std::collections::HashMap;
use std::time::{Duration, Instant};

/// Group key kind of a choke (vote kinds are Prevote 0 / Precommit 1).
const CHOKE_KIND: u8 = 2;

struct Held<T: Codec> {
    msg: OverlordMsg<T>,
    sig: Bytes,
    voter: Bytes,
    /// (height, round, vote_type, block_hash) of a vote; None for a choke
    vote: Option<(u64, u64, u8, Bytes)>,
    /// (height, round) of a choke
    choke: Option<(u64, u64)>,
    t: Instant,
}

/// Counters, as ingress.py `stats`.
#[derive(Clone, Debug, Default)]
pub struct IngressStats {
    pub batches: u64,
    pub prefetched: u64,
    pub forwarded: u64,
    pub dropped: u64,
    pub unbatched: u64,
}

/// `proc_network_msg` with vote batching. `forward` hands a decoded message to overlord
/// (`overlord_handler.send_msg(Context::new(), msg)`, consensus.rs:214-253).
pub struct VoteIngress<T: Codec, F: FnMut(OverlordMsg<T>)> {
    crypto: HipCrypto,
    forward: F,
    held: Vec<Held<T>>,
    groups: HashMap<(u64, u64, u8), usize>,
    /// None: the validator count (minus one for a validator), from `HipCrypto::pubkeys`
    pub batch_size: Option<usize>,
    pub max_delay: Duration,
    pub stats: IngressStats,
}

impl<T: Codec, F: FnMut(OverlordMsg<T>)> VoteIngress<T, F> {
    pub fn new(crypto: HipCrypto, forward: F) -> Self {
        VoteIngress {
            crypto,
            forward,
            held: Vec::new(),
            groups: HashMap::new(),
            batch_size: None,
            max_delay: Duration::from_millis(2),
            stats: IngressStats::default(),
        }
    }

    async fn limit(&self) -> usize {
        if let Some(b) = self.batch_size {
            return b.max(1);
        }
        let pks = self.crypto.pubkeys.read().await;
        if pks.is_empty() {
            return 256;
        }
        let own = pks.iter().any(|k| *k == self.crypto.name);
        (pks.len() - usize::from(own)).max(1)
    }

    /// consensus.rs:210-258: `msg_type` is `NetworkMsg::r#type`, `payload` its `msg`.
    pub async fn proc_network_msg(&mut self, msg_type: &str, payload: &[u8]) {
        self.poll().await; // the deadline of what is already held
        match msg_type {
            "SignedVote" => match rlp::decode::<SignedVote>(payload) {
                Ok(v) => {
                    let vt: u8 = v.vote.vote_type.clone().into();
                    let key = (v.vote.height, v.vote.round, vt);
                    let vote = Some((v.vote.height, v.vote.round, vt, v.vote.block_hash.clone()));
                    let (sig, voter) = (v.signature.clone(), v.voter.clone());
                    self.hold(OverlordMsg::SignedVote(v), key, sig, voter, vote, None).await;
                }
                Err(_) => self.drop_msg("decode SignedVote failed!"),
            },
            "SignedChoke" => match rlp::decode::<SignedChoke>(payload) {
                Ok(c) => {
                    let key = (c.choke.height, c.choke.round, CHOKE_KIND);
                    let choke = Some((c.choke.height, c.choke.round));
                    let (sig, addr) = (c.signature.clone(), c.address.clone());
                    self.hold(OverlordMsg::SignedChoke(c), key, sig, addr, None, choke).await;
                }
                Err(_) => self.drop_msg("decode SignedChoke failed!"),
            },
            "AggregatedVote" => match rlp::decode::<AggregatedVote>(payload) {
                Ok(a) => {
                    self.flush().await; // what arrived before goes first (arrival order)
                    self.send(OverlordMsg::AggregatedVote(a));
                }
                Err(_) => self.drop_msg("decode AggregatedVote failed!"),
            },
            "SignedProposal" => match rlp::decode::<SignedProposal<T>>(payload) {
                Ok(p) => {
                    self.flush().await;
                    self.send(OverlordMsg::SignedProposal(p));
                }
                Err(_) => self.drop_msg("decode SignedProposal failed!"),
            },
            _ => self.drop_msg("unexpected network msg!"),
        }
    }

    fn drop_msg(&mut self, why: &str) {
        eprintln!("overlord-hip ingress: {why}");
        self.stats.dropped += 1;
    }

    async fn hold(&mut self, msg: OverlordMsg<T>, key: (u64, u64, u8), sig: Bytes, voter: Bytes,
                  vote: Option<(u64, u64, u8, Bytes)>, choke: Option<(u64, u64)>) {
        self.held.push(Held { msg, sig, voter, vote, choke, t: Instant::now() });
        let c = self.groups.entry(key).or_insert(0);
        *c += 1;
        let full = *c >= self.limit().await;
        if full {
            self.flush().await;
        }
    }

    /// Flush when the oldest held message has waited `max_delay` (call from a timer).
    pub async fn poll(&mut self) {
        if self.held.first().map_or(false, |h| h.t.elapsed() >= self.max_delay) {
            self.flush().await;
        }
    }

    /// Batch-verify every held message (one `ovh_prefetch`, on a blocking task), then forward
    /// them in arrival order.
    pub async fn flush(&mut self) {
        let items = std::mem::take(&mut self.held);
        self.groups.clear();
        if items.is_empty() {
            return;
        }
        let keys: Vec<_> = items.iter().map(|h| (h.vote.clone(), h.choke)).collect();
        let sigs: Vec<Bytes> = items.iter().map(|h| h.sig.clone()).collect();
        let voters: Vec<Bytes> = items.iter().map(|h| h.voter.clone()).collect();
        let crypto = self.crypto.clone();
        // hashes and the prefetch block on the device: never on the reactor
        let res = tokio::task::spawn_blocking(move || {
            let hs = signed_hashes(&crypto, &keys);
            let fixed: Vec<usize> =
                (0..hs.len()).filter(|&k| sigs[k].len() == 96 && voters[k].len() == 48 && hs[k].len() == 32).collect();
            if fixed.is_empty() {
                return (0usize, hs.len());
            }
            let s: Vec<[u8; 96]> = fixed.iter().map(|&k| sigs[k].as_ref().try_into().unwrap()).collect();
            let h: Vec<[u8; 32]> = fixed.iter().map(|&k| hs[k].as_ref().try_into().unwrap()).collect();
            let p: Vec<[u8; 48]> = fixed.iter().map(|&k| voters[k].as_ref().try_into().unwrap()).collect();
            // a failed prefetch only costs cache misses: overlord's verify_signature still
            // checks every forwarded message on the device
            let _ = crypto.prefetch(&s, &h, &p);
            (fixed.len(), hs.len() - fixed.len())
        })
        .await;
        if let Ok((n, other)) = res {
            // other encodings go to overlord as they are: its verify_signature takes the exact
            // per-call path (a cache miss)
            self.stats.unbatched += other as u64;
            if n > 0 {
                self.stats.batches += 1;
                self.stats.prefetched += n as u64;
            }
        }
        for h in items {
            self.send(h.msg);
        }
    }

    fn send(&mut self, msg: OverlordMsg<T>) {
        self.stats.forwarded += 1;
        (self.forward)(msg);
    }
}

/// The signed hash of every held message: device vote digests for votes whose block hash
/// fits OVH_VOTE_HASH_MAX, Crypto::hash (SM3) of the RLP otherwise and for chokes.
fn signed_hashes(crypto: &HipCrypto, items: &[(Option<(u64, u64, u8, Bytes)>, Option<(u64, u64)>)]) -> Vec<Bytes> {
    use overlord::Crypto;
    let mut out: Vec<Option<Bytes>> = vec![None; items.len()];
    let idx: Vec<usize> = (0..items.len())
        .filter(|&i| matches!(&items[i].0, Some((_, _, _, bh)) if bh.len() <= ffi::OVH_VOTE_HASH_MAX))
        .collect();
    if !idx.is_empty() {
        let v = |i: usize| items[i].0.clone().unwrap();
        let hs: Vec<u64> = idx.iter().map(|&i| v(i).0).collect();
        let rs: Vec<u64> = idx.iter().map(|&i| v(i).1).collect();
        let ts: Vec<u8> = idx.iter().map(|&i| v(i).2).collect();
        let bs: Vec<Bytes> = idx.iter().map(|&i| v(i).3).collect();
        if let Ok(ds) = crypto.vote_digests(&hs, &rs, &ts, &bs) {
            for (k, &i) in idx.iter().enumerate() {
                out[i] = Some(Bytes::copy_from_slice(&ds[k]));
            }
        }
    }
    for (i, it) in items.iter().enumerate() {
        if out[i].is_some() {
            continue;
        }
        let mut s = rlp::RlpStream::new();
        match it {
            (Some((h, r, t, bh)), _) => {
                s.begin_list(4);
                s.append(h);
                s.append(r);
                s.append(t);
                s.append(&bh.to_vec());
            }
            (None, Some((h, r))) => {
                s.begin_list(2);
                s.append(h);
                s.append(r);
            }
            _ => unreachable!(),
        }
        out[i] = Some(crypto.hash(Bytes::from(s.out().to_vec())));
    }
    out.into_iter().map(|h| h.unwrap()).collect()
}
