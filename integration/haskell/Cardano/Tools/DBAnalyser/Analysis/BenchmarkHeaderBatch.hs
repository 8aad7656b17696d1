{-# LANGUAGE BangPatterns        #-}
{-# LANGUAGE RankNTypes          #-}
{-# LANGUAGE NamedFieldPuns      #-}
{-# LANGUAGE ScopedTypeVariables #-}

-- | A db-analyser analysis beside 'BenchmarkLedgerOps' (Analysis.hs:75-88, :479-607):
-- header revalidation of a Praos (Babbage/Conway) ImmutableDB in per-epoch batches on the
-- GPU through 'Ouroboros.Consensus.Protocol.Praos.Batch', timed per epoch the way
-- BenchmarkLedgerOps times per block (mutator ns), one line per epoch:
--
--   epoch  headers  validated  stop_verdict  ms  headers/s
--
-- A maintainer wires it in as one more 'AnalysisName' constructor
-- (@BenchmarkHeaderBatch (Maybe FilePath) Int@: output file, device) and one more
-- equation of runAnalysis (Analysis.hs:108-123).  The stream is the same
-- 'processAllImmutableDB' loop (Analysis.hs:815-847) with 'GetRawHeader' as the block
-- component, so the bytes the GPU decodes are exactly the stored header spans the
-- secondary index gives (Secondary.hs:93-128).  Shipped as source (no GHC here); the
-- ABI calls it makes are replayed from C by integration/c/ffi_harness.c.
module Cardano.Tools.DBAnalyser.Analysis.BenchmarkHeaderBatch
  ( benchmarkHeaderBatch
  , EpochBatchEnv (..)
  ) where

import           Control.Monad (unless, when)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Lazy as BSL
import           Data.IORef
import           Data.Word (Word64)
import qualified GHC.Stats as GC
import qualified System.IO as IO
import           Text.Printf (hPrintf)

import           Ouroboros.Consensus.Protocol.Praos.Batch

-- | What the analysis needs besides the stream: the epoch layout and stability window
-- (praosParams / EpochInfo), the ledger view (PoolDistr, envelope limits) installed per
-- epoch, the protocol parameters, and the genesis PraosState (CBOR).
data EpochBatchEnv = EpochBatchEnv
  { ebEpochInfo   :: (Word64, Word64, Word64, Word64)   -- base slot, base epoch, length, window
  , ebEnvLimits   :: (Word64, Word64, Word64, Word64)   -- maxMajorPV, pvMajor, maxHeaderSize, maxBodySize
  , ebPools       :: Word64 -> [(BS.ByteString, BS.ByteString, Integer)]   -- PoolDistr of an epoch
  , ebParams      :: PraosParamsC
  , ebStateCbor   :: BS.ByteString
  , ebDevice      :: Int
  }

-- | @benchmarkHeaderBatch out env stream@: @stream@ is the analysis' processAll over the
-- ImmutableDB with 'GetRawHeader' (slot and raw header bytes per block), folded here into
-- per-epoch batches.
benchmarkHeaderBatch
  :: Maybe FilePath
  -> EpochBatchEnv
  -> (forall st. st -> (st -> (Word64, BSL.ByteString) -> IO (Bool, st)) -> IO st)
  -> IO ()
benchmarkHeaderBatch mOut EpochBatchEnv {ebEpochInfo, ebEnvLimits, ebPools, ebParams, ebStateCbor, ebDevice}
                     stream =
  withOut mOut $ \h -> withPraosBatchCtx ebDevice $ \ctx -> do
    IO.hPutStrLn h "epoch\theaders\tvalidated\tstop_verdict\tms\theaders/s"
    stRef <- newIORef ebStateCbor
    tipRef <- newIORef Nothing
    let (base, baseNo, len, _) = ebEpochInfo
        epochOf s = baseNo + (s - base) `div` len
        -- one epoch's batch: tick, install the ledger view, validate, report
        flush _ [] = pure True
        flush e hdrsRev = do
          st <- readIORef stRef
          tip <- readIORef tipRef
          let hdrs = reverse hdrsRev
              firstSlot = fst (head hdrs)
          eta <- praosTickedEpochNonce st ebEpochInfo firstSlot
          praosSetEpoch ctx eta (ebPools e) ebParams
          t0 <- GC.mutator_elapsed_ns <$> GC.getRTSStats
          !r <- praosValidateHeaderBytes ctx ebEpochInfo ebEnvLimits tip st (map snd hdrs)
          t1 <- GC.mutator_elapsed_ns <$> GC.getRTSStats
          let n = length hdrs
              ms = fromIntegral (t1 - t0) / 1e6 :: Double
              stopped = brChainStop r < n
              verdict = if stopped then brVerdicts r !! brChainStop r else 0
          hPrintf h "%d\t%d\t%d\t%d\t%.3f\t%.0f\n" e n (brChainStop r) verdict ms
                  (fromIntegral n / max 1e-9 (ms / 1e3))
          writeIORef stRef (brState r)
          writeIORef tipRef (brTip r)
          pure (not stopped)          -- the reference stops at the first invalid header
    (e, acc, ok) <- stream (0, [], True) $ \(e, acc, ok) (slot, raw) -> do
      let e' = epochOf slot
          hdr = (slot, BSL.toStrict raw)
      if null acc || e' == e
        then pure (True, (e', hdr : acc, ok))
        else do
          ok' <- flush e acc
          pure (ok', (e', [hdr], ok'))
    when ok $ do
      _ <- flush e acc
      pure ()
    unless ok $ IO.hPutStrLn h "# stopped at the first invalid header"
  where
    withOut (Just f) k = IO.withFile f IO.WriteMode k
    withOut Nothing k = k IO.stdout
